#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: every rank on cuda:0, gloo instead of RCCL
# (RFRT_BENCH_ONE_GPU=1; never used for reported numbers).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp RFRT_BENCH_ONE_GPU=1
for n in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 1 > gpurun_out/bench_rehearse_$n.log 2>&1; rc=$?; tail -2 gpurun_out/bench_rehearse_$n.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
done
