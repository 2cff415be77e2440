#!/bin/bash
# GPU-box: host-path parity tests, then host-path rate vs chunk size with small runs moved by
# kernel (LSEC_KERNEL_COPY=1) vs the default policy (small runs packed), alternating processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "host or pageable or fn_pointer or segment or verify or file_tools or magic" > gpurun_out/pytest_kcopy.log 2>&1 || exit 1
echo "pytest ok"
for rep in 1 2; do
  export LSEC_KERNEL_COPY=1
  timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_ab.txt 2>&1 || exit 1
  unset LSEC_KERNEL_COPY
  timeout -k 10 300 python tools/host_chunk_ab.py "$@" >> gpurun_out/kcopy_ab.txt 2>&1 || exit 1
done
echo done
