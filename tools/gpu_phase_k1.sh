#!/bin/bash
# GPU box: the XCD tile phase (third field: 0 off, 1 tile loops, 3 also the networks) on the
# large-chunk encodes (RS at C = 4 / 8 MiB, Cauchy at 8 MiB, the headline), interleaved in one
# allocation per configuration.  (Run r06j also A/B'ed plain against non-temporal loads and stores
# through a fourth field, since removed: no shape moved, profiles/r06_v10_tile_phase_mem_mode_ab.txt.)
#   gpurun -- bash tools/gpu_phase_k1.sh <tag>
set -o pipefail
tag=${1:-phk1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/phase_k1_${tag}.txt
timeout -k 10 900 python tools/kbench.py --configs rs84c8,rs104c8,rs164c8,rs63c8,rs84c4,cg164c8,cg206c8,rs63 \
  --variants "0,0,0;0,0,1;0,0,3" --rounds 7 --data-gib 16 > $o 2>&1 || { echo "kbench failed"; tail -5 $o; exit 1; }
grep variant $o
