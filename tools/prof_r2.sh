#!/bin/bash
# rocprofv3 passes over one bench.py command (no CPU baseline): kernel trace + stats, then one PMC
# pass per counter group, each in its own run (gfx950: FETCH_SIZE and WRITE_SIZE cannot share a
# pass; no other trace domain beside --pmc).  Output: gpurun_out/prof_${TAG}/<pass>/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/prof_${TAG}
ARGS=${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
PASSES=${PASSES:-"stats;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"}
mkdir -p $OUT
IFS=';' read -ra G <<< "$PASSES"
i=0
for g in "${G[@]}"; do
  if [ "$g" = "stats" ]; then
    timeout -k 10 ${PT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o k -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
  else
    timeout -s KILL ${PT:-300} rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/p$i -o k -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  fi
  rc=$?
  echo "pass $i ($g) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/*.log; exit $rc; }
  i=$((i+1))
done
find $OUT -name '*.csv' | head -30
exit 0
