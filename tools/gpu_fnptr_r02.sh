#!/bin/bash
# GPU box: LStore's per-stripe fn-pointer call pattern (tools/fnptr_bench.c), engine vs the
# reference (oracle/_ref) on the same host threads, chunk x threads x path.
#   gpurun -- bash tools/gpu_fnptr_r02.sh <tag> [chunks] [threads]
set -o pipefail
tag=${1:-run}
chunks=${2:-"16384 65536 1048576"}
threads=${3:-"1 8 32 128"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out="gpurun_out/fnptr_${tag}.jsonl"
: > "$out"
REF="$PWD/oracle/_ref/libjerasure_ref.so"
for C in $chunks; do
  for T in $threads; do
    calls=${SECS:-2}
    for method in cauchy_good reed_sol_van; do
      FNPTR_REF=$REF timeout -k 10 120 build/fnptr_bench $C $T $calls $method encode >> "$out" || { echo "fail C=$C T=$T $method"; exit 1; }
      LSEC_SMALL_PATH=dispatch timeout -k 10 120 build/fnptr_bench $C $T $calls $method encode >> "$out" || { echo "fail dispatch C=$C T=$T"; exit 1; }
      FNPTR_PINNED=1 timeout -k 10 120 build/fnptr_bench $C $T $calls $method encode >> "$out" || { echo "fail pinned C=$C T=$T"; exit 1; }
    done
    FNPTR_REF=$REF timeout -k 10 120 build/fnptr_bench $C $T $calls cauchy_good decode >> "$out" || { echo "fail decode C=$C T=$T"; exit 1; }
  done
done
echo "fnptr ok: $(wc -l < "$out") lines"
