#!/bin/bash
# GPU-box: kernel-transport host path (LSEC_KERNEL_COPY=1) by copy-kernel grid size, plus the
# packing default, one process per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/kcopy_grid.txt
for g in 64 256 1024 4096; do
  echo "# LSEC_COPY_GRID=$g" >> gpurun_out/kcopy_grid.txt
  LSEC_KERNEL_COPY=1 LSEC_COPY_GRID=$g timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_grid.txt 2>&1 || exit 1
done
echo "# default (packing)" >> gpurun_out/kcopy_grid.txt
timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_grid.txt 2>&1 || exit 1
echo done
