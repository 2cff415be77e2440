#!/bin/bash
# GPU box: per-stripe calls above the zero-copy limit, concurrency-gated own pipeline (default)
# vs always the dispatcher (LSEC_OWN_PIPELINE_MAX=0), alternating processes (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/route_1m2.jsonl; : > $out
for rep in 1 2; do
  for cfg in "1048576 reed_sol_van encode" "1048576 cauchy_good decode" "524288 reed_sol_van encode" "524288 cauchy_good decode"; do
    set -- $cfg
    for T in 1 8 32; do
      timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 $3 | sed "s/^{/{\"route\": \"gated\", \"rep\": $rep, /" >> $out || { echo "fail $cfg T=$T"; exit 1; }
      LSEC_OWN_PIPELINE_MAX=0 timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 $3 | sed "s/^{/{\"route\": \"dispatcher\", \"rep\": $rep, /" >> $out || { echo "fail d $cfg T=$T"; exit 1; }
    done
  done
done
echo ok
