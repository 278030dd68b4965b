cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_coverage.py tests/test_gpu_dist_tracer.py -m gpu > gpurun_out/pt_cov.log 2>&1; rc=$?; tail -15 gpurun_out/pt_cov.log; [ $rc -eq 0 ] || exit $rc
SHARDS=1,8 timeout -k 10 400 python -u tools/cov_profile.py > gpurun_out/covprof.log 2>&1; rc=$?; grep case gpurun_out/covprof.log; [ $rc -eq 0 ] || exit $rc
CASES=k3,k5 SHARDS=1,8 REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c2 -o kt -- python3 tools/cov_profile.py > gpurun_out/prof_c2.log 2>&1
