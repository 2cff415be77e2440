#!/bin/bash
# GPU box: per-stripe decode_block calls (Cauchy-good(6+3), lost D0) at 16 / 64 KiB and 8 / 32 /
# 128 threads with LSEC_STATS phase means and wait counters (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_decode.txt; : > $out
for C in 16384 65536; do
  for T in 8 32 128; do
    echo "== decode $C cauchy_good T=$T" >> $out
    LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench $C $T 2 cauchy_good decode >> $out 2>&1 || { echo "fail C=$C T=$T"; exit 1; }
  done
done
echo ok
