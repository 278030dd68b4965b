mkdir -p gpurun_out
RFRT_BVH_PACKET=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coverage.py tests/test_gpu_fullsize.py -k "bvh or k4 or terrain or k5" -v -x --timeout 300 --timeout-method thread > gpurun_out/r6i_pytest_packet.txt 2>&1 || exit 1
SCENE=terrain VAR_ENV=RFRT_BVH_PACKET VARIANTS="0 1 0 1" timeout -k 10 400 python -u tools/trace_variants.py > gpurun_out/r6i_trace_packet.jsonl 2>&1 || exit 1
LIBS="rf_ray_tracing_warp_amd/librfrt.so rf_ray_tracing_warp_amd/librfrt.so@RFRT_BVH_PACKET=1" CASES=k5 REPS=5 timeout -k 10 400 python -u tools/cov_variants.py > gpurun_out/r6i_cov_packet.jsonl 2>&1
