#!/bin/bash
# Round-end style check on one GPU: the whole -m gpu suite, smoke(), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.txt; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 280 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1; rc2=$?
tail -c 200 gpurun_out/${TAG}_bench.log; exit $((rc + rc2))
