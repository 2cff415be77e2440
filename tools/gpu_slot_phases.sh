#!/bin/bash
# Phase times of the own-slot zero-copy route (LSEC_STATS=1) for per-stripe calls of one size,
# under each environment given: gpurun -- bash tools/gpu_slot_phases.sh <tag> <chunk> <threads> <method> <op> "ENV=V[,ENV=V]" ...
set -o pipefail
tag=$1; chunk=$2; threads=$3; method=$4; op=$5
shift 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/slot_phases_${tag}.txt
: > "$out"
for envs in "$@"; do
  echo "== $envs" >> "$out"
  env LSEC_STATS=1 ${envs//,/ } timeout -k 10 60 build/fnptr_bench "$chunk" "$threads" 3 "$method" "$op" >> "$out" 2>&1 \
    || { echo "failed: $envs"; tail -5 "$out"; exit 1; }
done
grep -E "^==|own-slot|server calls|gibps" "$out" | sed 's/"per_call_us_p99.*"gibps"/ ... "gibps"/' | cut -c1-300
