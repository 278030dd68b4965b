#!/bin/bash
# round-2 GPU session: new parity/poison/device tests first (verbose, per-test timeout), then the
# whole GPU suite.  Stops at a crash-like status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r2}
ok() { case "$1" in 0|1|5) return 0;; *) echo "STOP: status $1" ; return 1;; esac; }
timeout -k 10 ${T1:-900} python -u -m pytest ${FIRST:-tests/test_gpu_poison.py tests/test_gpu_fullsize.py tests/test_gpu_dist_tracer.py} -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -30 gpurun_out/${TAG}_new.log; ok $rc || exit $rc
[ -n "$NO_ALL" ] && exit 0
timeout -k 10 ${T2:-900} python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -15 gpurun_out/${TAG}_all.log; exit $rc
