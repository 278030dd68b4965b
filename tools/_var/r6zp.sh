set -o pipefail
TAG=r6zp T_TESTS=600 bash tools/gpu.sh tests smoke bench rehearse || exit 1
MODE=sectors TAG=r6zp bash tools/gpu.sh ranks timeline
