#!/bin/bash
# c5 lows, round 5: bytewise shapes of the device lows (tools/kbench.py), and host-path calls
# repeated over one buffer (tools/host_reps.py) for the host lows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/lows2; mkdir -p "$O"
timeout -k 10 600 python tools/kbench.py --configs rs84c8,rs124c4,cg206c2,rs63 --variants "0,0;1,0;2,0;3,0;4,0;5,0" --rounds 3 --data-gib 12 \
  > "$O/kbench_lows.txt" 2>&1 || { echo "kbench failed"; tail -5 "$O/kbench_lows.txt"; exit 1; }
echo "ok kbench"
for cfg in "reed_sol_van 20 6 4194304" "reed_sol_van 6 3 1048576" "cauchy_good 8 4 524288" "reed_sol_van 4 2 262144"; do
  set -- $cfg
  LSEC_TRACE=1 timeout -k 10 200 python tools/host_reps.py --method $1 --k $2 --m $3 --chunk $4 --reps 6 > "$O/host_$1_$2_$3_$4.jsonl" 2> "$O/host_$1_$2_$3_$4.trace" || { echo "host reps failed $cfg"; exit 1; }
done
echo "ok host reps"
