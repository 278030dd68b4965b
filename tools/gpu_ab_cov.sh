#!/bin/bash
# Coverage replay A/B on one GPU: the coverage parity tests (poison + oracle), then K3/K5 maps timed
# and hashed with the receiver-first replay on (default) and off (RFRT_COV_RXFIRST=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 ${T1:-600} python -u -m pytest ${TESTS:-tests/test_gpu_poison.py tests/test_gpu_coverage.py} -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.txt; case $rc in 0|1) ;; *) exit $rc;; esac
L=rf_ray_tracing_warp_amd/librfrt.so
CASES=${CASES:-k3,k5} LIBS="$L@RFRT_COV_RXFIRST=0 $L $L@RFRT_COV_RXFIRST=0 $L" timeout -k 10 ${T2:-500} python -u tools/cov_variants.py > gpurun_out/${TAG}_cov.jsonl 2>&1
rc2=$?; cat gpurun_out/${TAG}_cov.jsonl; exit $((rc + rc2))
