#!/bin/bash
# GPU box: GPU tests + smoke, then LStore's per-stripe fn-pointer table, engine vs the reference
# on the same host threads (tools/gpu_fnptr_r02.sh).
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "gpurun_out/pytest_gpu_${tag}.txt" 2>&1 \
  || { echo "gpu tests failed"; tail -30 "gpurun_out/pytest_gpu_${tag}.txt"; exit 1; }
echo "gpu tests ok: $(tail -1 gpurun_out/pytest_gpu_${tag}.txt)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_${tag}.txt" 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke ok"
timeout -k 10 700 bash tools/gpu_fnptr_r02.sh "${tag}" || exit 1
