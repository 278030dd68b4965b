#!/bin/bash
# Coverage A/B against tools/_var/lib_*.so: coverage parity tests on librfrt.so first, then K3/K5 maps
# timed + hashed per library, then the rank-of-8 estimate per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-cab}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_coverage.py tests/test_gpu_poison.py tests/test_gpu_fullsize.py} -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.txt; [ $rc -ne 0 ] && exit $rc
L=rf_ray_tracing_warp_amd/librfrt.so
V=$(ls tools/_var/lib_*.so | tr '\n' ' ')
CASES=k3,k5 LIBS="$L $V $L $V" timeout -k 10 400 python -u tools/cov_variants.py > gpurun_out/${TAG}_cov.jsonl 2>&1 || exit $?
cat gpurun_out/${TAG}_cov.jsonl
for lib in $L $V; do
  RFRT_LIB_PATH=$lib SHARDS=8 REPS=3 timeout -k 10 200 python -u tools/cov_profile.py > gpurun_out/${TAG}_ranks_$(basename $lib .so).jsonl 2>&1 || exit $?
  echo $lib; grep '"shards": 8' gpurun_out/${TAG}_ranks_$(basename $lib .so).jsonl | cut -c1-200
done
