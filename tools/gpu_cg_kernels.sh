#!/bin/bash
# GPU box: Cauchy w = 8 encodes on the compiled packet network (variant 0,0) against the generic
# bit-sliced kernel at 1 / 2 / 4 dwords per lane (0,1 / 0,2 / 0,4), every c5 (k, m) at C = 1, 4, 8 MiB,
# interleaved in one allocation per shape (tools/kbench.py).
#   gpurun -- bash tools/gpu_cg_kernels.sh <tag>
set -o pipefail
tag=${1:-cgk}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/cg_kernels_${tag}.txt
timeout -k 10 1000 python tools/kbench.py --configs cg:4:2:1024,cg:4:2:4096,cg:4:2:8192,cg:6:3:1024,cg:6:3:4096,cg:6:3:8192,cg:8:3:1024,cg:8:3:4096,cg:8:3:8192,cg:8:4:1024,cg:8:4:4096,cg:8:4:8192,cg:10:4:1024,cg:10:4:4096,cg:10:4:8192,cg:12:4:1024,cg:12:4:4096,cg:12:4:8192,cg:16:4:1024,cg:16:4:4096,cg:16:4:8192,cg:20:6:1024,cg:20:6:4096,cg:20:6:8192 \
  --variants "0,0;0,1;0,2;0,4" --rounds 5 --data-gib 12 > $o 2>&1 || { echo "kbench failed"; tail -5 $o; exit 1; }
grep variant $o
