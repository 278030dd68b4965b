set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6zk_pytest.txt 2>&1; tail -n1 gpurun_out/r6zk_pytest.txt
TAG=r6zk LIBS="tools/_var/lib_reg0.so rf_ray_tracing_warp_amd/librfrt.so tools/_var/lib_reg2.so tools/_var/lib_reg8.so tools/_var/lib_reg0.so rf_ray_tracing_warp_amd/librfrt.so" bash tools/ab_lib_trace.sh > gpurun_out/r6zk_ab.log 2>&1; grep -v cells gpurun_out/r6zk_ab.log | grep sectors | cut -c1-150
