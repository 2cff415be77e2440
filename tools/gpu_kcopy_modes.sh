#!/bin/bash
# GPU-box: host path by transport mode, alternating processes: packing default, LSEC_KERNEL_COPY=1
# (kernel in, DMA out), =2 (kernel both ways).  Then the host-path parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/kcopy_modes.txt
for rep in 1 2; do
  for mode in 0 1 2; do
    if [ $mode = 0 ]; then unset LSEC_KERNEL_COPY; else export LSEC_KERNEL_COPY=$mode; fi
    timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_modes.txt 2>&1 || exit 1
  done
done
unset LSEC_KERNEL_COPY
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "small_runs" \
    > gpurun_out/pytest_modes.log 2>&1 || exit 1
echo done
