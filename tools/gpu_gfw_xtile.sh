#!/bin/bash
# GPU box: the w = 16 / 32 network tests, then kbench of the RS networks with and without the
# cross-tile input prefetch (LSEC_JIT_VARIANT bit 19), alternating processes.
#   gpurun -- bash tools/gpu_gfw_xtile.sh <tag>
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gfw_network or wide_fields" > "gpurun_out/gfw_pytest_${tag}.txt" 2>&1 || { tail -30 "gpurun_out/gfw_pytest_${tag}.txt"; exit 1; }
tail -1 "gpurun_out/gfw_pytest_${tag}.txt"
out="gpurun_out/gfw_xtile_${tag}.txt"
: > "$out"
for round in 1 2; do
  for v in 0 0x80000; do
    echo "== round $round variant $v" >> "$out"
    LSEC_JIT_VARIANT=$v timeout -k 10 300 python tools/kbench.py --configs rs63w32,rs104w32,rs104w16,rs206w16 --variants "0,0" \
      --rounds 3 2>&1 | grep -v amdgpu.ids >> "$out" || { echo "kbench failed"; tail "$out"; exit 1; }
  done
done
cat "$out"
