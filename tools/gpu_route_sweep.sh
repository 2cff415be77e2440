#!/bin/bash
# GPU-box: per-stripe calls (tools/fnptr_bench.c, 4x-LLC working set) over chunk sizes and thread
# counts under route variants; one JSON line each in gpurun_out/route_<tag>.jsonl.
#   gpurun -- bash tools/gpu_route_sweep.sh <tag> "<chunks>" "<threads>" "<method:op ...>" "ENV=V ..." ...
set -o pipefail
tag=$1; chunks=$2; threads=$3; ops=$4; shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/route_${tag}.jsonl; : > "$out"
for c in $chunks; do for t in $threads; do for mo in $ops; do
  IFS=: read -r method op <<< "$mo"
  for v in "$@"; do
    env $v FNPTR_SET_MB=2048 timeout -k 10 60 build/fnptr_bench "$c" "$t" 1.5 "$method" "$op" | sed "s/}\$/, \"env\": \"$v\"}/" >> "$out" || exit 1
  done
  env FNPTR_ONLY_REF=1 FNPTR_REF=oracle/_ref/libjerasure_ref.so FNPTR_SET_MB=2048 timeout -k 10 60 build/fnptr_bench "$c" "$t" 1.5 "$method" "$op" | sed "s/}\$/, \"env\": \"reference\"}/" >> "$out" || exit 1
done; done; echo "done $c"; done
