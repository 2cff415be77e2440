#!/bin/bash
# HBM channel-spread probe: RS(6+3) / Cauchy(10+4) encode + decode with padding after every shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for pad in 0 256 4096 12288 65536 0; do
  echo "pad=$pad" >> gpurun_out/kb_pad.log
  timeout -k 10 200 python tools/kbench.py --configs rs63,cg104 --variants "0,0" --rounds 3 --pad $pad 2>&1 | grep -v amdgpu >> gpurun_out/kb_pad.log || exit 1
done
echo done
