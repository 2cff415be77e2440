#!/bin/bash
# GPU box: the XCD tile phase and the memory-instruction mode (4th field: 1 plain stores, 2 plain
# loads, 3 both) on the large-chunk encodes (RS at C = 4 / 8 MiB, Cauchy at 8 MiB, the headline),
# phase off / on interleaved in one allocation per configuration, 9 rounds.
#   gpurun -- bash tools/gpu_phase_k1.sh <tag>
set -o pipefail
tag=${1:-phk1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/phase_k1_${tag}.txt
timeout -k 10 900 python tools/kbench.py --configs rs84c8,rs104c8,rs164c8,rs63c8,rs84c4,cg164c8,cg206c8,rs63 \
  --variants "0,0,0,0;0,0,1,0;0,0,0,1;0,0,0,2;0,0,0,3" --rounds 7 --data-gib 16 > $o 2>&1 || { echo "kbench failed"; tail -5 $o; exit 1; }
grep variant $o
