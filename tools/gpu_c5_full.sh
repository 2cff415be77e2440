#!/bin/bash
# GPU box: the whole c5 sweep (tools/sweep.py: 8 (k, m) x 6 chunk sizes x 2 methods, device-resident
# and host path, every point bit-exact), one (method, k+m) group per step with its own time limit;
# summary by tools/sweep_summary.py.
#   gpurun --timeout 1200 -- bash tools/gpu_c5_full.sh <tag> [methods]   (one method per call fits the limit)
set -o pipefail
tag=${1:-c5}
methods=${2:-"reed_sol_van cauchy_good"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/sweep_c5_${tag}.jsonl
for meth in $methods; do
  for km in 4+2 6+3 8+3 8+4 10+4 12+4 16+4 20+6; do
    timeout -k 10 240 python tools/sweep.py --methods $meth --km $km --out $o > gpurun_out/sweep_c5_${tag}_${meth}_${km}.log 2>&1 \
      || { echo "sweep failed: $meth $km"; tail -5 gpurun_out/sweep_c5_${tag}_${meth}_${km}.log; exit 1; }
    echo "ok $meth $km ($(wc -l < $o) points)"
  done
done
python tools/sweep_summary.py $o > gpurun_out/sweep_c5_${tag}_summary.txt && cat gpurun_out/sweep_c5_${tag}_summary.txt
