#!/bin/bash
# GPU box: small-call A/B, current build vs HEAD's (build/oldlib), 3 alternating reps of the
# configurations where the two differed (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/futex_ab2.jsonl; : > $out; : > gpurun_out/futex_routes2.txt
for rep in 1 2 3; do
  for cfg in "16384 reed_sol_van 1" "16384 reed_sol_van 32" "16384 reed_sol_van 128" "65536 reed_sol_van 32" "65536 reed_sol_van 128" "65536 reed_sol_van 256" "65536 cauchy_good 128" "65536 cauchy_good 256"; do
    set -- $cfg
    LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench $1 $3 2 $2 encode 2>gpurun_out/futex_stats.txt | sed "s/^{/{\"build\": \"new\", \"rep\": $rep, /" >> $out || { echo "fail new $cfg"; exit 1; }
    echo "$cfg $(cat gpurun_out/futex_stats.txt)" >> gpurun_out/futex_routes2.txt
    LD_LIBRARY_PATH=$PWD/build/oldlib timeout -k 10 60 build/fnptr_bench $1 $3 2 $2 encode | sed "s/^{/{\"build\": \"head\", \"rep\": $rep, /" >> $out || { echo "fail old $cfg"; exit 1; }
  done
done
echo "ok $(wc -l < $out)"
