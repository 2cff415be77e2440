#!/bin/bash
# GPU box: per-phase means and wait counters (LSEC_STATS=1) of pageable 16 KiB RS(6+3)
# encode_block calls at 32 / 64 / 128 threads (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_phases3.txt; : > $out
for T in 32 64 128 128; do
  echo "== 16384 reed_sol_van T=$T" >> $out
  LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 $T 2 reed_sol_van encode >> $out 2>&1 || { echo "fail T=$T"; exit 1; }
done
echo "== 16384 reed_sol_van T=128 LSEC_WAIT_POLLERS=1" >> $out
LSEC_WAIT_POLLERS=1 LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 128 2 reed_sol_van encode >> $out 2>&1 || exit 1
echo "== 16384 reed_sol_van T=128 LSEC_WAIT_SPINNERS=0" >> $out
LSEC_WAIT_SPINNERS=0 LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 128 2 reed_sol_van encode >> $out 2>&1 || exit 1
echo ok
