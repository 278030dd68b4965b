set -o pipefail
TAG=r6zi T_TESTS=600 bash tools/gpu.sh tests smoke bench rehearse || exit 1
MODE=sectors TAG=r6zi bash tools/gpu.sh ranks timeline
