#!/bin/bash
# GPU box: GPU tests, then host-path A/B of LSEC_KERNEL_COPY (unset vs 1) at small chunks with
# the round-2 pinning threshold (tools/pin_run_ab.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r02_v27.txt 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu_r02_v27.txt; exit 1; }
echo "gpu tests ok: $(tail -1 gpurun_out/pytest_gpu_r02_v27.txt)"
timeout -k 10 400 python -u tools/pin_run_ab.py --env LSEC_KERNEL_COPY --settings=-,1 --chunks 16384,65536,131072,262144,524288 --gib 0.75 \
  > gpurun_out/kcopy_ab.jsonl 2> gpurun_out/kcopy_ab.err && echo kcopy-ok
