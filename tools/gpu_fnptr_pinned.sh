#!/bin/bash
# GPU-box: dispatcher parity tests, then the LStore fn-pointer call pattern on page-locked
# buffers (FNPTR_PINNED=1), copy-piece kernel (default) vs per-request DMA (LSEC_KERNEL_COPY=0),
# alternating processes.  build/fnptr_bench is built on the CPU side (see tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "fn_pointer or concurrent or device_set or segment" > gpurun_out/pytest_fnpin.log 2>&1 || exit 1
echo "pytest ok"
: > gpurun_out/fnptr_pinned.txt
export FNPTR_PINNED=1
for rep in 1 2; do
  for chunk in 16384 65536 262144; do
    for t in 8 32; do
      unset LSEC_KERNEL_COPY
      timeout -k 10 120 ./build/fnptr_bench $chunk $t 48 reed_sol_van >> gpurun_out/fnptr_pinned.txt 2>&1 || exit 1
      LSEC_KERNEL_COPY=0 timeout -k 10 120 ./build/fnptr_bench $chunk $t 48 reed_sol_van >> gpurun_out/fnptr_pinned.txt 2>&1 || exit 1
    done
  done
done
echo done
