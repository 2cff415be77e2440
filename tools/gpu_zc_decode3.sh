#!/bin/bash
# GPU box: pageable 16 KiB Cauchy-good(6+3) decode_block at 128 threads, repeated (does the
# throttled regime recur?), and 16 KiB encodes beside it (LSEC_STATS=1; tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_decode3.txt; : > $out
for rep in 1 2; do
  for op in decode encode; do
    echo "== $op rep $rep" >> $out
    LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 128 2 cauchy_good $op >> $out 2>&1 || { echo "fail $op"; exit 1; }
  done
done
echo "== decode 256 threads" >> $out
LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 256 2 cauchy_good decode >> $out 2>&1 || exit 1
echo ok
