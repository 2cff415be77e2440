#!/bin/bash
# GPU box: small-call and pointer tests, then the per-phase means of tools/gpu_zc_phases.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/phases2_pytest.txt 2>&1 || { echo "tests failed"; tail -20 gpurun_out/phases2_pytest.txt; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/phases2_pytest.txt)"
timeout -k 10 500 bash tools/gpu_zc_phases.sh
