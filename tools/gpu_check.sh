#!/bin/bash
# GPU-box check used with gpurun: parity tests, then the headline bench under rocprofv3.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag> [pytest -k expression]
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
tag=${1:-run}
sel=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${sel:+-k "$sel"} \
    > "gpurun_out/pytest_${tag}.log" 2>&1 && echo "pytest ok" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_${tag}" -o run -- \
    python bench.py > "gpurun_out/bench_${tag}.log" 2>&1 && echo "bench ok"
