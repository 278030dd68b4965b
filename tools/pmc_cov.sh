#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, kernel trace only) over tools/cov_profile.py
# (CASES/SHARDS/REPS from the environment).  Output: gpurun_out/pmc_${TAG}/g<i>/...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-cov}
OUT=gpurun_out/pmc_${TAG}
GROUPS_=${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY;GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY"}
mkdir -p $OUT
i=0
IFS=';' read -ra G <<< "$GROUPS_"
for g in "${G[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/g$i -o k -- python3 tools/cov_profile.py > $OUT/g$i.log 2>&1
  rc=$?
  echo "group $i ($g) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
