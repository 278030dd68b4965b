#!/bin/bash
# Coverage GPU check: coverage/full-size/poison/distributed tests, rank-of-8 projection,
# K3/K5 map timings + hashes, and one rocprofv3 kernel trace of a K3 + K5 map.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-cc}
timeout -k 10 700 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_fullsize.py tests/test_gpu_poison.py \
  tests/test_gpu_dist_tracer.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/cov_profile.py > gpurun_out/${TAG}_cov_ranks.jsonl 2>&1 || exit $?
cut -c1-220 gpurun_out/${TAG}_cov_ranks.jsonl
CASES=k3,k5 LIBS=rf_ray_tracing_warp_amd/librfrt.so timeout -k 10 300 python -u tools/cov_variants.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o k -- \
  python3 tools/cov_variants.py child k3,k5 1 > gpurun_out/${TAG}_trace.log 2>&1
