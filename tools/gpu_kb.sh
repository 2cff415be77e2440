#!/bin/bash
# GPU-box: parity tests, kernel A/B bench over the c5 RS/Cauchy shapes, headline bench under rocprofv3.
#   gpurun --timeout 1200 -- bash tools/gpu_kb.sh <tag>
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "gpurun_out/pytest_${tag}.log" 2>&1 && echo "pytest ok" && \
timeout -k 10 600 python tools/kbench.py --configs rs206,rs164,rs124,rs104,rs84,rs63,cg104,cg63 --variants "0,0" \
    --rounds 3 --magic > "gpurun_out/kb_${tag}.log" 2>&1 && echo "kbench ok" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_${tag}" -o run -- \
    python bench.py > "gpurun_out/bench_${tag}.log" 2>&1 && echo "bench ok"
