#!/bin/bash
# One rocprofv3 --pmc pass per counter group (kernel trace only, no other trace domains) over a
# bench.py command.  PMC_GROUPS is a ';'-separated list of space-separated counter groups.
# Output: gpurun_out/pmc_${TAG}/g<i>/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/pmc_${TAG}
ARGS=${PMC_ARGS:---steps 5 --warmup 1 --no-cpu-baseline --no-coverage --no-k4}
GROUPS_=${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_INSTS_LDS SQ_INSTS_BRANCH;SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY;GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY"}
mkdir -p $OUT
i=0
IFS=';' read -ra G <<< "$GROUPS_"
for g in "${G[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/g$i -o k -- python3 bench.py $ARGS > $OUT/g$i.log 2>&1
  rc=$?
  echo "group $i ($g) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
