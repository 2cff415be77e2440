#!/bin/bash
# Registered zero-copy route (LSEC_REG_ZC=1) reproducer: tools/reg_stress.py for SECONDS per case
# with host-array churn and stripe-server calls mixed in, under each environment given.
#   gpurun -- bash tools/gpu_reg_repro.sh <tag> <seconds> "ENV=V[,ENV=V]" ...
# GEOS="<reg_stress args>;<reg_stress args>" replaces the two default geometries; REGZC=0 takes
# the default routes instead of the registered one.
set -o pipefail
tag=${1:-run}
secs=${2:-30}
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/reg_repro_${tag}.jsonl
: > "$out"
for envs in "$@"; do
  IFS=';' read -ra geos <<< "${GEOS:---k 6 --m 3 --w 16 --chunk 49192;--method cauchy_good --k 6 --m 3 --chunk 65536 --stripes 1}"
  for geo in "${geos[@]}"; do
    env LSEC_REG_ZC=${REGZC:-1} ${envs//,/ } timeout -k 10 $((secs + 60)) python tools/reg_stress.py --seconds "$secs" --churn --small-mix $geo \
      | sed "s/}\$/, \"env\": \"$envs\"}/" >> "$out" || { echo "failed: $envs $geo"; exit 1; }
    tail -1 "$out" | cut -c1-400
  done
done
