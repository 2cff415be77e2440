#!/bin/bash
# GPU box: per-stripe calls of 1-4 MiB (RS(6+3) at 128 / 256 KiB chunks): the dispatcher
# (default) vs a zero-copy launch of the call's own (LSEC_ZEROCOPY_KB=4096), alternating
# processes, every call verified against oracle/_ref (tools/fnptr_bench.c FNPTR_VERIFY=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/route_mid.jsonl; : > $out
export FNPTR_VERIFY=1 FNPTR_REF=$PWD/oracle/_ref/libjerasure_ref.so
for rep in 1 2; do
  for C in 131072 262144; do
    for op in encode decode; do
      for T in 1 8 32 128; do
        timeout -k 10 60 build/fnptr_bench $C $T 2 reed_sol_van $op | sed "s/^{/{\"route\": \"dispatcher\", \"rep\": $rep, /" >> $out || { echo "fail $C $op T=$T"; exit 1; }
        LSEC_ZEROCOPY_KB=4096 timeout -k 10 60 build/fnptr_bench $C $T 2 reed_sol_van $op | sed "s/^{/{\"route\": \"zerocopy\", \"rep\": $rep, /" >> $out || { echo "fail zc $C $op T=$T"; exit 1; }
      done
    done
  done
done
echo ok
