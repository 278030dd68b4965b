cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_coverage.py tests/test_gpu_dist_tracer.py -m gpu > gpurun_out/pt_cov.log 2>&1; rc=$?; tail -3 gpurun_out/pt_cov.log; [ $rc -eq 0 ] || exit $rc
export MODE=rays REPS=2
for c in k3 k5; do
  for s in 1 8; do
    CASES=$c SHARDS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cov_${c}_${s} -o k -- python3 tools/cov_profile.py > gpurun_out/prof_cov_${c}_${s}.log 2>&1 || exit 1
  done
done
grep -h case gpurun_out/prof_cov_*.log
