#!/bin/bash
# GPU box: the C = 8 MiB encode dip against an occupancy cap (LSEC_WGS_CAP = workgroups per CU, as
# unused dynamic LDS; occupancy_lds_bytes in ec_kernels.hip): the c5 lows' encodes at C = 1 and 8 MiB,
# equal bytes per launch, for every cap.  One kbench run per cap, each with its own time limit.
#   gpurun -- bash tools/gpu_wgs_cap.sh <tag> [caps...]
set -o pipefail
tag=${1:-wgs}
shift
caps=${*:-"0 2 3 4 6"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/wgs_cap_${tag}.txt
: > $o
for c in $caps; do
  echo "== LSEC_WGS_CAP=$c" >> $o
  LSEC_WGS_CAP=$c timeout -k 10 240 python tools/kbench.py --configs rs84,rs84c8,cg164c1,cg164c8,cg206c1,cg206c8 --variants "0,0" \
    --rounds 3 --data-gib 20 >> $o 2>&1 || { echo "kbench failed at cap $c"; tail -5 $o; exit 1; }
done
grep -E "==|variant" $o
