cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pt_all.log 2>&1; rc=$?; tail -5 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
TAG=r1c bash tools/profile.sh > gpurun_out/profile_r1c.log 2>&1 || exit 1
export MODE=rays REPS=2
for c in k3 k5; do
  for s in 1 8; do
    CASES=$c SHARDS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cov_${c}_${s} -o k -- python3 tools/cov_profile.py > gpurun_out/prof_cov_${c}_${s}.log 2>&1 || exit 1
  done
done
grep -h case gpurun_out/prof_cov_*.log
