#!/bin/bash
# GPU-box: kernel-transport tests, then caller-pinned / pageable host rates with and without
# LSEC_KERNEL_COPY=1, alternating processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "small_runs or host or pinned" \
    > gpurun_out/pytest_kpinned.log 2>&1 || exit 1
echo "pytest ok"
: > gpurun_out/kcopy_pinned.txt
for rep in 1 2; do
  LSEC_KERNEL_COPY=1 timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_pinned.txt 2>&1 || exit 1
  timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_pinned.txt 2>&1 || exit 1
done
echo done
