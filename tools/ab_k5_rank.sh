#!/bin/bash
# K5 rank-of-8 A/B over variant libraries (run on the GPU box from the repo root):
#   gpurun -- 'TAG=r3za LIBS="..." bash tools/ab_k5_rank.sh'
# For every library: the full-size K5 8-rank bit-identity test (ray-sharded map == whole map), then
# tools/cov_profile.py's K5 rank projection -> gpurun_out/${TAG}_k5_rank_ab.jsonl.  Stops at the
# first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}_k5_rank_ab.jsonl
: > $O
for lib in ${LIBS:-rf_ray_tracing_warp_amd/librfrt.so}; do
  b=$(basename $lib .so)
  RFRT_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_fullsize.py -k "k5_ray_sharded" -m gpu > gpurun_out/${TAG:-ab}_${b}_k5test.txt 2>&1
  rc=$?; echo "$b test rc=$rc: $(tail -1 gpurun_out/${TAG:-ab}_${b}_k5test.txt)"
  [ $rc -ne 0 ] && exit $rc
  RFRT_LIB_PATH=$lib CASES=k5 SHARDS=8 timeout -k 10 300 python -u tools/cov_profile.py 2>/dev/null | \
    sed "s/^{/{\"lib\": \"$b\", /" >> $O
  rc=$?; [ $rc -ne 0 ] && exit $rc
  tail -1 $O | cut -c1-250
done
exit 0
