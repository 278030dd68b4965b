#!/bin/bash
# rocprofv3 passes over bench.py (no CPU baseline): kernel trace + stats, then one PMC pass per
# TCC counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Output: gpurun_out/prof_${TAG}/{trace,fetch,write}/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/prof_${TAG}
ARGS=${PROF_ARGS:---steps 20 --warmup 3 --no-cpu-baseline}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o k -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o k -- python3 bench.py $ARGS > $OUT/write.log 2>&1
rc=$?; echo "profile rc=$rc"; find $OUT -name '*.csv' | head -20; exit $rc
