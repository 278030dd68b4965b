#!/bin/bash
# A/B of BVH traversal variant libraries (tools/_var/lib_*.so vs librfrt.so): K4 trace and K5
# coverage timings + output hashes.  Stops at the first crash-like status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-var}
LIBS=${LIBS:-"rf_ray_tracing_warp_amd/librfrt.so $(ls tools/_var/lib_*.so | tr '\n' ' ')"}
SCENE=terrain LIBS="$LIBS" timeout -k 10 ${T1:-400} python -u tools/trace_variants.py > gpurun_out/${TAG}_trace.jsonl 2>&1
rc=$?; cat gpurun_out/${TAG}_trace.jsonl; case $rc in 0|3) ;; *) exit $rc;; esac
[ -n "$NO_COV" ] && exit 0
CASES=${CASES:-k5} LIBS="$LIBS" timeout -k 10 ${T2:-500} python -u tools/cov_variants.py > gpurun_out/${TAG}_cov.jsonl 2>&1
rc=$?; cat gpurun_out/${TAG}_cov.jsonl; exit $rc
