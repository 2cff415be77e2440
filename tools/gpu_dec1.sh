#!/bin/bash
# GPU-box: per-stripe 1 MiB calls (tools/fnptr_bench.c, 4x-LLC working set) under route variants,
# one JSON line each in gpurun_out/dec1_<tag>.jsonl.   gpurun -- bash tools/gpu_dec1.sh <tag> "ENV=V ..." ...
set -o pipefail
tag=${1:-run}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/dec1_${tag}.jsonl; : > "$out"
for v in "$@"; do
  for c in "1048576 1 2 cauchy_good decode" "1048576 8 2 cauchy_good decode" "1048576 1 2 reed_sol_van encode" "1048576 8 2 reed_sol_van encode" "262144 1 2 cauchy_good decode"; do
    env $v FNPTR_SET_MB=2048 timeout -k 10 60 build/fnptr_bench $c | sed "s/}\$/, \"env\": \"$v\"}/" >> "$out" || exit 1
  done
done
