#!/bin/bash
# GPU box: 16 KiB Cauchy-good(6+3) decode_block at 8 and 128 threads, encode at 128, with the
# LSEC_STATS counters (runtime pointer queries per call) (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_decode4.txt; : > $out
for cfg in "8 decode" "128 decode" "128 encode"; do
  set -- $cfg
  echo "== $2 T=$1" >> $out
  LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 $1 2 cauchy_good $2 >> $out 2>&1 || { echo "fail $cfg"; exit 1; }
done
echo ok
