#!/bin/bash
# GPU-box: LStore's per-stripe call pattern (tools/fnptr_bench.c) with every thread walking its own
# stripes over a working set of 4x the host's last-level caches (FNPTR_SET_MB default), engine
# and reference (oracle/_ref) alike.  One JSON line per run in gpurun_out/fnptr_fair_<tag>.jsonl.
#   gpurun -- bash tools/gpu_fnptr_fair.sh <tag> ["chunk:threads:method:op[:ENV=V]" ...]
set -o pipefail
tag=${1:-run}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/fnptr_fair_${tag}.jsonl
: > "$out"
cases=${*:-"1048576:1:cauchy_good:decode 1048576:8:cauchy_good:decode 65536:8:cauchy_good:decode 65536:1:cauchy_good:decode 16384:1:cauchy_good:decode 16384:8:cauchy_good:decode"}
for c in $cases; do
  IFS=: read -r chunk threads method op envs <<< "$c"
  for impl in engine reference; do
    # the harness's own settings (FNPTR_*: buffer lifetime, page-locked buffers) apply to both
    # sides, the engine's (LSEC_*) to the engine only
    harness=""
    for e in ${envs//,/ }; do case $e in FNPTR_*) harness="$harness $e" ;; esac; done
    if [ $impl = reference ]; then extra="FNPTR_ONLY_REF=1$harness"; else extra="${envs//,/ }"; fi
    env FNPTR_REF=oracle/_ref/libjerasure_ref.so $extra timeout -k 10 60 build/fnptr_bench "$chunk" "$threads" 2 "$method" "$op" \
      | sed "s/}\$/, \"env\": \"$extra\"}/" >> "$out" || { echo "failed: $c $impl"; exit 1; }
  done
  echo "done $c"
done
