cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pt_all.log 2>&1; rc=$?; tail -5 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
GS=8 timeout -k 10 300 python -u tools/bvh_steps.py > gpurun_out/bvh_steps.log 2>&1; rc=$?; grep mode gpurun_out/bvh_steps.log; [ $rc -eq 0 ] || exit $rc
SHARDS=1,8 timeout -k 10 400 python -u tools/cov_profile.py > gpurun_out/covprof.log 2>&1; rc=$?; grep case gpurun_out/covprof.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
