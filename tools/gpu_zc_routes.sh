#!/bin/bash
# GPU box: which route LStore's per-stripe encode_block calls take (LSEC_STATS=1 counters) at
# 8 / 32 / 128 threads, tools/fnptr_bench.c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_routes.txt; : > $out
for cfg in "65536 cauchy_good" "65536 reed_sol_van" "16384 cauchy_good" "16384 reed_sol_van"; do
  set -- $cfg
  for T in 8 32 128; do
    echo "== $1 $2 T=$T" >> $out
    LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode >> $out 2>&1 || { echo "fail $cfg T=$T"; exit 1; }
  done
done
echo ok
