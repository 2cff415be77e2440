#!/bin/bash
# GPU box: the XCD tile phase on the bytewise kernel's large-chunk encodes (RS at C = 4 / 8 MiB),
# phase off / on interleaved in one allocation per configuration, 9 rounds.
#   gpurun -- bash tools/gpu_phase_k1.sh <tag>
set -o pipefail
tag=${1:-phk1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/phase_k1_${tag}.txt
timeout -k 10 900 python tools/kbench.py --configs rs84c8,rs83c8,rs104c8,rs164c8,rs63c8,rs84c4,rs124c4,rs104c4 \
  --variants "0,0,0;0,0,1" --rounds 9 --data-gib 16 > $o 2>&1 || { echo "kbench failed"; tail -5 $o; exit 1; }
grep variant $o
