#!/bin/bash
# Registered zero-copy route (LSEC_REG_ZC=1) under caller buffers at several alignments: each
# case a separate process, every byte of every call checked against the oracle restatement.
#   gpurun --timeout 900 -- bash tools/gpu_reg_probe.sh <tag> [iters]
set -o pipefail
tag=${1:-run}
iters=${2:-30}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out="gpurun_out/reg_probe_${tag}.jsonl"
: > "$out"
export LSEC_REG_ZC=${LSEC_REG_ZC:-1}
for off in -1 0 16 48 528 4080; do
  for geo in "--k 20 --m 6 --w 8" "--k 10 --m 4 --w 16" "--k 6 --m 3 --w 32 --chunk 262144" \
             "--k 6 --m 3 --w 8 --chunk 1048576 --stripes 1 --method cauchy_good"; do
    timeout -k 10 120 python tools/reg_stress.py --iters "$iters" --offset "$off" $geo >> "$out" 2> "gpurun_out/reg_probe_${tag}.err" \
      || { echo "reg_stress failed: off=$off $geo"; tail -20 "gpurun_out/reg_probe_${tag}.err"; exit 1; }
  done
done
cat "$out"
