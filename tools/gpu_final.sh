#!/bin/bash
# GPU-box: headline bench under rocprofv3 (kernel trace + stats), then the PMC traffic passes.
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_${tag}" -o run -- \
    python bench.py > "gpurun_out/bench_${tag}.log" 2>&1 && echo "bench ok" && \
timeout -k 10 600 python tools/pmc_traffic.py "${tag}" > "gpurun_out/pmc_${tag}.log" 2>&1 && echo "pmc ok"
