#!/bin/bash
# GPU box: which per-stripe cases trip the in-place stall guard (stderr per case), verified calls,
# 10 s each: the 1 MiB encode at three threads with long-lived buffers and with LStore's freed
# buffers (FNPTR_FREE_AFTER=1, glibc's heap), twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/guard_cases.jsonl; : > $out
export FNPTR_VERIFY=1 FNPTR_REF=$PWD/oracle/_ref/libjerasure_ref.so
for rep in 1 2; do
  for fa in 0 1; do
    err=$(FNPTR_FREE_AFTER=$fa timeout -k 10 60 build/fnptr_bench 1048576 3 10 reed_sol_van encode 2>&1 >> $out) \
      || { echo "FAIL free_after=$fa"; exit 1; }
    echo "rep $rep free_after=$fa: guard trips $(echo "$err" | grep -c stalled)"
  done
done
