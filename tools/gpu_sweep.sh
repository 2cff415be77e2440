#!/bin/bash
# GPU box: config c5 sweep (tools/sweep.py) on the current build.
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/sweep.py --methods reed_sol_van,cauchy_good --out "gpurun_out/sweep_c5_${tag}.jsonl" > "gpurun_out/sweep_${tag}.log" 2>&1 || { echo "sweep failed"; tail -20 "gpurun_out/sweep_${tag}.log"; exit 1; }
echo "sweep ok"
