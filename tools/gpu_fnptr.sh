#!/bin/bash
# GPU-box: the unmodified LStore call pattern (tools/fnptr_bench.c, built on the CPU side into build/)
#   gpurun --timeout 900 -- bash tools/gpu_fnptr.sh <tag>
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for chunk in 16384 65536 1048576; do
  for t in 1 8 32 128; do
    calls=$(( chunk >= 1048576 ? 16 : 48 ))
    timeout -k 10 120 ./build/fnptr_bench $chunk $t $calls cauchy_good >> "gpurun_out/fnptr_${tag}.txt" 2>&1 || exit 1
  done
done
echo done
