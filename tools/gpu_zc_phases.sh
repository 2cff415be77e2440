#!/bin/bash
# GPU box: where a per-stripe encode_block call's wall time goes (LSEC_STATS=1 phase means),
# tools/fnptr_bench.c at 1 / 8 / 32 / 128 threads, pageable and page-locked callers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_phases.txt; : > $out
for cfg in "16384 reed_sol_van" "65536 reed_sol_van"; do
  set -- $cfg
  for pin in 0 1; do
    for T in 1 8 32 128; do
      echo "== $1 $2 T=$T pinned=$pin" >> $out
      FNPTR_PINNED=$pin LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode >> $out 2>&1 || { echo "fail $cfg T=$T"; exit 1; }
    done
  done
done
echo ok
