#!/bin/bash
# K2 A/B (librfrt.so vs tools/_var/lib_*.so, alternated): step and trace-kernel times + output hashes,
# then the trace parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-k2ab}
L=rf_ray_tracing_warp_amd/librfrt.so
V=$(ls tools/_var/lib_*.so | tr '\n' ' ')
LIBS="$L $V $L $V" timeout -k 10 300 python -u tools/k2_fused_variants.py > gpurun_out/${TAG}_k2.jsonl 2>&1 || exit $?
cat gpurun_out/${TAG}_k2.jsonl
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_trace_cir.py} -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.txt; exit $rc
