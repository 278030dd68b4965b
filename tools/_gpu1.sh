cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_coverage.py -m gpu > gpurun_out/pt_cov.log 2>&1; rc=$?; tail -5 gpurun_out/pt_cov.log; [ $rc -eq 0 ] || exit $rc
CASES=k3,k5 SHARDS=1,8 MODE=rays timeout -k 10 300 python -u tools/cov_profile.py > gpurun_out/covprof_rays.log 2>&1 || exit 1
CASES=k3,k5 SHARDS=8 MODE=cells timeout -k 10 300 python -u tools/cov_profile.py > gpurun_out/covprof_cells.log 2>&1 || exit 1
RFRT_COV_FUSED=1 CASES=k3 SHARDS=1 timeout -k 10 300 python -u tools/cov_profile.py > gpurun_out/covprof_fused.log 2>&1 || exit 1
grep -h case gpurun_out/covprof_*.log
