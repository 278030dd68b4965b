mkdir -p gpurun_out/prof_r6h
i=0
for g in "TA_BUSY_avr TA_BUSY_max" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LEVEL_WAVES" "GRBM_GUI_ACTIVE GRBM_TA_BUSY" "TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d gpurun_out/prof_r6h/p$i -o k -- python3 tools/k4_write_ab.py > gpurun_out/prof_r6h/p$i.log 2>&1 || exit 1
  i=$((i+1))
done
