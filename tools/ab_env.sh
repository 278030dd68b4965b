# A/B of one runtime switch on the rank projection: ENVVAR, VALUES (space separated), TAG
set -o pipefail
mkdir -p gpurun_out
for v in ${VALUES}; do
  env ${ENVVAR}=$v MODE=${MODE:-sectors} CASES=${CASES:-k3,k5} timeout -k 10 200 python -u tools/cov_profile.py > gpurun_out/${TAG}_ab_$v.jsonl 2>&1 || exit 1
  echo "${ENVVAR}=$v"; cut -c1-170 gpurun_out/${TAG}_ab_$v.jsonl | grep -v cells
done
