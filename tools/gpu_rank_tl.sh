#!/bin/bash
# Kernel timeline of one ray-shard rank-pass (rank 7 of 8) for K3 and K5: rocprofv3 --kernel-trace
# over tools/cov_profile.py, then tools/rank_timeline.py on each trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-tl}
for c in ${CASES:-k3 k5}; do
  CASES=$c SHARDS=8 REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$c -- python3 tools/cov_profile.py > gpurun_out/${TAG}_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_$c.log
  python3 tools/rank_timeline.py gpurun_out/${TAG}_$c > gpurun_out/${TAG}_$c.timeline.txt || exit $?
  cat gpurun_out/${TAG}_$c.timeline.txt
done
