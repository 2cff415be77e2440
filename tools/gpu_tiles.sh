#!/bin/bash
# Work-sharing tiles on the box (ec_kernels.h "Work-sharing tiles"): the three tile modes A/B'd on
# the headline (tools/tiles_ab.py), the static prefix's share varied, per-XCD finish times of the
# engine's own kernels (tools/xcd_stamps.py), and the tile-mode parity tests.
#   gpurun -- bash tools/gpu_tiles.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-t}; O=gpurun_out/tiles_$tag; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 python tools/tiles_ab.py --trials 4 --json "$O/tiles_ab.jsonl" > "$O/tiles_ab.log" 2>&1 || { echo "tiles_ab failed"; tail -5 "$O/tiles_ab.log"; exit 1; }
echo "ok tiles_ab"
for pre in 48 60; do
  LSEC_TILES_PRE_64THS=$pre timeout -k 10 300 python tools/tiles_ab.py --trials 2 --json "$O/tiles_ab_pre$pre.jsonl" > "$O/tiles_ab_pre$pre.log" 2>&1 || { echo "tiles_ab pre $pre failed"; exit 1; }
done
echo "ok pre"
timeout -k 10 300 python tools/xcd_stamps.py --trials 2 --json "$O/xcd_stamps.jsonl" > "$O/xcd_stamps.log" 2>&1 || { echo "stamps failed"; exit 1; }
echo "ok stamps"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k tile_sharing > "$O/pytest_tiles.txt" 2>&1; tail -2 "$O/pytest_tiles.txt"
