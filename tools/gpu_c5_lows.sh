#!/bin/bash
# The c5 points furthest below their rooflines, each swept alone with the
# host path's phase trace (LSEC_TRACE=1: pin / submit / drain / unpin per host call) and the PCIe
# link fractions (tools/sweep.py).  Device: RS(8+4) 8 MiB encode, RS(12+4) 4 MiB decode,
# Cauchy-good(20+6) 2 MiB decode.  Host: RS(20+6) 4 MiB, RS(4+2) 256 KiB, Cauchy-good(8+4) 512 KiB,
# and the headline RS(6+3) 1 MiB for reference.
#   gpurun -- bash tools/gpu_c5_lows.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-lows}
O=gpurun_out/c5_$tag; mkdir -p "$O"
for pt in "reed_sol_van 8+4 8388608" "reed_sol_van 12+4 4194304" "cauchy_good 20+6 2097152" \
          "reed_sol_van 20+6 4194304" "reed_sol_van 4+2 262144" "cauchy_good 8+4 524288" "reed_sol_van 6+3 1048576"; do
  set -- $pt
  name="$1_$2_$(( $3 >> 10 ))k"
  LSEC_TRACE=1 timeout -k 10 300 python tools/sweep.py --methods "$1" --km "$2" --chunks "$3" --out "$O/sweep.jsonl" \
    > "$O/$name.log" 2> "$O/$name.trace" || { echo "failed $name"; tail -5 "$O/$name.trace"; exit 1; }
  echo "ok $name"
done
