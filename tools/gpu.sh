#!/bin/bash
# The one GPU-session driver (run on the box through gpurun):
#
#   gpurun --timeout 1200 -- 'TAG=r3a bash tools/gpu.sh full'
#
# Every task writes under gpurun_out/${TAG}_* (copy what is judged into profiles/, see
# profiles/README.md).  Each GPU step has its own time limit; the script stops at the first
# failing step (a failed test may be a GPU fault that Python caught), so a faulting kernel never
# gets a second launch in one call.  CONTINUE=1 lets the next step run after ordinary test
# failures (pytest rc 1 / 5) only; crash-like statuses (abort, segfault, time limit) always stop.
#
# tasks (space-separated, run in order):
#   tests     pytest ${TESTS:-tests} -m gpu (verbose, per-test timeout)     -> ${TAG}_pytest_gpu.txt
#   smoke     __graft_entry__.smoke()                                        -> ${TAG}_smoke.txt
#   bench     python bench.py ${BENCH_ARGS}                                  -> ${TAG}_bench.log / .json
#   stats     rocprofv3 --kernel-trace --stats over bench.py ${PROF_ARGS}    -> prof_${TAG}/stats
#   pmc       one rocprofv3 --pmc pass per group of ${PASSES} over bench.py  -> prof_${TAG}/p<i>
#   ranks     tools/cov_profile.py (K3/K5, 1 and 8 ray-shard ranks)          -> ${TAG}_cov_ranks.jsonl
#   timeline  rocprofv3 kernel trace of one rank-of-8 pass (TL_SHARDS=1: the whole map) + rank_timeline -> ${TAG}_<case>.timeline.txt
#   covvar    tools/cov_variants.py over LIBS (A/B, hashed)                  -> ${TAG}_cov.jsonl
#   tracevar  tools/trace_variants.py over LIBS (SCENE=room|terrain)         -> ${TAG}_trace.jsonl
#   k2var     tools/k2_fused_variants.py over LIBS                           -> ${TAG}_k2.jsonl
#   k4write   rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE over tools/k4_write_ab.py, per library in LIBS
#   ossort    tools/os_sort_bench vs rocPRIM (built on the box)               -> ${TAG}_os_sort.jsonl
#   rehearse  bench.py N=2,4 on this one GPU (gloo, RFRT_BENCH_ONE_GPU=1)    -> ${TAG}_rehearse_<n>.log
#   full      = tests smoke bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/${TAG}
L=rf_ray_tracing_warp_amd/librfrt.so
LIBS=${LIBS:-"$L $(ls tools/_var/lib_*.so 2>/dev/null | tr '\n' ' ')"}

step_rc() {  # $1 status, $2 name: 0 continue, else stop the script with that status
  case "$1" in
    0) return 0 ;;
    1|5) echo "$2: rc=$1 (failures)"; [ -z "$CONTINUE" ] && exit "$1"; return 0 ;;
    *) echo "STOP after $2: status $1"; exit "$1" ;;
  esac
}

run_task() {
  case "$1" in
    tests)
      timeout -k 10 ${T_TESTS:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -v -x --timeout ${T_TEST:-400} \
        --timeout-method thread > ${O}_pytest_gpu.txt 2>&1
      rc=$?; tail -4 ${O}_pytest_gpu.txt; step_rc $rc tests ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1
      rc=$?; tail -2 ${O}_smoke.txt; step_rc $rc smoke ;;
    bench)
      timeout -k 10 ${T_BENCH:-400} python -u bench.py ${BENCH_ARGS} > ${O}_bench.log 2>&1
      rc=$?; tail -1 ${O}_bench.log > ${O}_bench.json; tail -c 400 ${O}_bench.log; echo; step_rc $rc bench ;;
    stats)
      mkdir -p gpurun_out/prof_${TAG}
      timeout -k 10 ${T_PROF:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}/stats \
        -o k -- python3 bench.py ${PROF_ARGS:---steps 20 --warmup 3 --no-cpu-baseline} > gpurun_out/prof_${TAG}/stats.log 2>&1
      rc=$?; echo "stats rc=$rc"; step_rc $rc stats ;;
    pmc)
      # gfx950: FETCH_SIZE and WRITE_SIZE each take their own pass; no other trace domain beside --pmc
      mkdir -p gpurun_out/prof_${TAG}
      IFS=';' read -ra G <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH}"
      i=0
      for g in "${G[@]}"; do
        timeout -s KILL ${T_PMC:-240} rocprofv3 --pmc $g --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}/p$i \
          -o k -- python3 ${PMC_CMD:-bench.py ${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}} > gpurun_out/prof_${TAG}/p$i.log 2>&1
        rc=$?; echo "pmc pass $i ($g) rc=$rc"; step_rc $rc "pmc $g"
        i=$((i + 1))
      done ;;
    ranks)
      timeout -k 10 ${T_RANKS:-300} python -u tools/cov_profile.py > ${O}_cov_ranks.jsonl 2>&1
      rc=$?; cut -c1-260 ${O}_cov_ranks.jsonl; step_rc $rc ranks ;;
    timeline)
      for c in ${CASES:-k3 k5}; do
        CASES=$c SHARDS=${TL_SHARDS:-8} REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ${O}_tl_$c -- \
          python3 tools/cov_profile.py > ${O}_tl_$c.log 2>&1
        rc=$?; step_rc $rc "timeline $c"
        python3 tools/rank_timeline.py ${O}_tl_$c > ${O}_$c.timeline.txt; tail -30 ${O}_$c.timeline.txt
      done ;;
    covvar)
      CASES=${CASES:-k3,k5} LIBS="$LIBS" timeout -k 10 ${T_VAR:-500} python -u tools/cov_variants.py > ${O}_cov.jsonl 2>&1
      rc=$?; cat ${O}_cov.jsonl | cut -c1-300; step_rc $rc covvar ;;
    tracevar)
      SCENE=${SCENE:-terrain} LIBS="$LIBS" timeout -k 10 ${T_VAR:-400} python -u tools/trace_variants.py > ${O}_trace.jsonl 2>&1
      rc=$?; cat ${O}_trace.jsonl | cut -c1-300; case $rc in 3) rc=0 ;; esac; step_rc $rc tracevar ;;
    k2var)
      LIBS="$LIBS" timeout -k 10 ${T_VAR:-300} python -u tools/k2_fused_variants.py > ${O}_k2.jsonl 2>&1
      rc=$?; cat ${O}_k2.jsonl | cut -c1-300; step_rc $rc k2var ;;
    k4write)
      # WRITE_SIZE / FETCH_SIZE of k_trace_bvh<5> per output set, for every library in LIBS
      mkdir -p gpurun_out/prof_${TAG}
      for lib in $LIBS; do
        b=$(basename $lib .so)
        for c in WRITE_SIZE FETCH_SIZE; do
          RFRT_LIB_PATH=$lib timeout -s KILL ${T_PMC:-180} rocprofv3 --pmc $c --kernel-trace --output-format csv \
            -d gpurun_out/prof_${TAG}/k4w_${b}_$c -o k -- python3 tools/k4_write_ab.py > gpurun_out/prof_${TAG}/k4w_${b}_$c.log 2>&1
          rc=$?; echo "k4write $b $c rc=$rc"; tail -1 gpurun_out/prof_${TAG}/k4w_${b}_$c.log | cut -c1-300; step_rc $rc "k4write $b"
        done
      done ;;
    ossort)
      # tool binaries are not pushed (.gpurunignore): build on the box, same image; one per digit width
      for b in ${OS_BITS_LIST:-8 10 12}; do
        timeout -k 10 300 hipcc -O3 --offload-arch=gfx950 -std=c++17 -DOS_BITS=$b tools/os_sort_bench.hip -o /tmp/os_sort_bench$b
        rc=$?; step_rc $rc "ossort build $b"
        for a in "786432 35 0.5" "1048576 30 0.5" "200000 30 0.5" "6291456 36 0.3"; do
          timeout -k 10 60 /tmp/os_sort_bench$b $a >> ${O}_os_sort.jsonl 2>&1
          rc=$?; tail -1 ${O}_os_sort.jsonl; step_rc $rc "ossort $b $a"
        done
      done ;;
    rehearse)
      for n in 2 4; do
        RFRT_BENCH_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 1 > ${O}_rehearse_$n.log 2>&1
        rc=$?; tail -1 ${O}_rehearse_$n.log | cut -c1-600; step_rc $rc "rehearse $n"
      done ;;
    full) run_task tests; run_task smoke; run_task bench ;;
    *) echo "unknown task $1"; exit 2 ;;
  esac
}

for t in "$@"; do run_task "$t"; done
exit 0
