# Per library in LIBS (or per value of ENVVAR in VALUES): tools/cov_profile.py (one-GPU maps + rank
# plans) under rocprofv3 --kernel-trace; tools/trace_case_kernels.py splits the traces per case
set -o pipefail
i=0
for x in ${LIBS:-${VALUES}}; do
  if [ -n "${LIBS}" ]; then e="RFRT_LIB_PATH=$x"; else e="${ENVVAR}=$x"; fi
  env $e MODE=${MODE:-sectors} SHARDS=${SHARDS:-1,8} REPS=${REPS:-2} CASES=${CASES:-k3,k5} timeout -k 10 300 rocprofv3 \
    --kernel-trace --output-format csv -d gpurun_out/${TAG}_lib$i -o k -- python3 tools/cov_profile.py \
    > gpurun_out/${TAG}_lib$i.jsonl 2>&1 || exit 1
  echo "lib$i: $e"; grep sectors gpurun_out/${TAG}_lib$i.jsonl | cut -c1-150
  i=$((i + 1))
done
