#!/bin/bash
# GPU-box: LStore's per-stripe calls (tools/fnptr_bench.c, FNPTR_VERIFY=1: every call's outputs
# overwritten before it and compared with oracle/_ref after it) on the registered zero-copy
# route's sizes, each case for SECONDS.  One JSON line per case in gpurun_out/reg_verify_<tag>.jsonl.
#   gpurun -- bash tools/gpu_reg_verify.sh <tag> [seconds] [ENV=V ...]
set -o pipefail
tag=${1:-run}
secs=${2:-5}
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/reg_verify_${tag}.jsonl
: > "$out"
for kv in "$@"; do export "${kv?}"; done
for c in 1048576:1:cauchy_good:decode 1048576:2:cauchy_good:decode 1048576:8:cauchy_good:decode \
         1048576:1:reed_sol_van:encode 1048576:4:reed_sol_van:encode 524288:1:cauchy_good:decode \
         524288:2:reed_sol_van:encode 2097152:1:cauchy_good:decode; do
  IFS=: read -r chunk threads method op <<< "$c"
  FNPTR_VERIFY=1 FNPTR_REF=oracle/_ref/libjerasure_ref.so timeout -k 10 $((secs + 60)) \
    build/fnptr_bench "$chunk" "$threads" "$secs" "$method" "$op" >> "$out"
  rc=$?
  tail -1 "$out" | cut -c1-220
  [ $rc -eq 0 ] || [ $rc -eq 2 ] || { echo "failed ($rc): $c"; exit 1; }
done
