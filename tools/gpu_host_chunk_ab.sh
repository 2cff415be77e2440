#!/bin/bash
# GPU-box: host-path rate vs chunk size, in-place pinning vs packing, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  unset LSEC_NO_HOST_REGISTER
  timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/host_chunk_ab.txt 2>&1 || exit 1
  export LSEC_NO_HOST_REGISTER=1
  timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/host_chunk_ab.txt 2>&1 || exit 1
done
echo done
