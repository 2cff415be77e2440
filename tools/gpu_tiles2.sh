#!/bin/bash
# Round-5 follow-up: tile modes with one body call site (tools/tiles_ab.py), the tile parity tests,
# and fresh allocations by torch vs the VMM API in 64 MiB / 256 MiB / 1 GiB physical pieces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/tiles_e; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k tile_sharing > "$O/pytest_tiles.txt" 2>&1 || { tail -20 "$O/pytest_tiles.txt"; exit 1; }
tail -1 "$O/pytest_tiles.txt"
timeout -k 10 400 python tools/tiles_ab.py --trials 4 --json "$O/tiles_ab.jsonl" > "$O/tiles_ab.log" 2>&1 || { echo "tiles_ab failed"; tail -5 "$O/tiles_ab.log"; exit 1; }
echo "ok tiles_ab"
timeout -k 10 900 python tools/alloc_pmc_probe.py --trials 16 --alloc torch,vmm:64,vmm:256,vmm:1024 \
  --json "$O/alloc_chunks.jsonl" > "$O/alloc_chunks.log" 2>&1 || { echo "alloc chunks failed"; tail -5 "$O/alloc_chunks.log"; exit 1; }
echo "ok alloc chunks"
