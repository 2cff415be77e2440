#!/bin/bash
# GPU box: the XCD tile phase A/B (lsec_test_set_tile_phase; ec_kernels.h) on the c5 lows and the
# headline, each configuration one allocation with the phase off / on interleaved (tools/kbench.py
# variants "0,0,0" and "0,0,3": off, and on for the tile loops and the networks; run r06g passed 1 when
# that meant both), after the bit-identity test.
#   gpurun -- bash tools/gpu_phase_ab.sh <tag>
set -o pipefail
tag=${1:-phase}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tile_phase" --timeout 120 --timeout-method thread \
  > gpurun_out/phase_test_${tag}.txt 2>&1 || { echo "phase test failed"; tail -20 gpurun_out/phase_test_${tag}.txt; exit 1; }
tail -1 gpurun_out/phase_test_${tag}.txt
o=gpurun_out/phase_ab_${tag}.txt
timeout -k 10 600 python tools/kbench.py --configs rs84c8,cg164c8,cg206c8,rs84,cg164c1,cg206c1,rs63,rs104c8 \
  --variants "0,0,0;0,0,3" --rounds 5 --data-gib 16 > $o 2>&1 || { echo "kbench failed"; tail -5 $o; exit 1; }
grep variant $o
