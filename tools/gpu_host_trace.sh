#!/bin/bash
# GPU-box: LSEC_TRACE phase times of the host path (pin / submit / drain / unpin) for the
# packing default, kernel transport and pinned-in-place DMA.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/host_trace.txt
echo "# default" >> gpurun_out/host_trace.txt
LSEC_TRACE=1 timeout -k 10 300 python tools/host_chunk_ab.py --chunks 262144,1048576 --reps 1 >> gpurun_out/host_trace.txt 2>&1 || exit 1
echo "# LSEC_KERNEL_COPY=1" >> gpurun_out/host_trace.txt
LSEC_TRACE=1 LSEC_KERNEL_COPY=1 timeout -k 10 300 python tools/host_chunk_ab.py --chunks 262144 --reps 1 >> gpurun_out/host_trace.txt 2>&1 || exit 1
echo done
