#!/bin/bash
# GPU session helper: parity tests, then bench. Stops on a crash/timeout-like status (not on
# ordinary test failures, rc 1), so a faulting kernel never gets a second launch in one call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { case "$1" in 0|1|5) return 0;; *) echo "STOP: status $1" ; return 1;; esac; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
if [ -n "$NO_BENCH" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; exit $rc
