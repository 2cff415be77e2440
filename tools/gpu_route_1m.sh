#!/bin/bash
# GPU box: per-stripe calls of 1 MiB chunks (9 MiB per RS(6+3) stripe: above the zero-copy
# limit), dispatcher (default) vs the in-place-pinned host pipeline (LSEC_COALESCE_MB=0),
# alternating processes (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/route_1m.jsonl; : > $out
for rep in 1 2; do
  for cfg in "reed_sol_van encode" "cauchy_good decode" "cauchy_good encode"; do
    set -- $cfg
    for T in 1 8 32; do
      timeout -k 10 60 build/fnptr_bench 1048576 $T 2 $1 $2 | sed "s/^{/{\"route\": \"dispatcher\", \"rep\": $rep, /" >> $out || { echo "fail $cfg T=$T"; exit 1; }
      LSEC_COALESCE_MB=0 timeout -k 10 60 build/fnptr_bench 1048576 $T 2 $1 $2 | sed "s/^{/{\"route\": \"host-pipeline\", \"rep\": $rep, /" >> $out || { echo "fail hp $cfg T=$T"; exit 1; }
    done
  done
done
echo ok
