#!/bin/bash
# Pinned-DMA copy shapes (tools/probes/rect_probe.cpp) at the c5 host lows, and the tile modes
# A/B'd at the c5 device lows (tools/tiles_ab.py).
set -o pipefail
O=gpurun_out/rect; mkdir -p $O
for pt in "8 3 524288 256" "8 4 524288 256" "4 2 1048576 256" "16 4 262144 256" "8 3 262144 512" "8 3 4194304 32"; do
  timeout -k 10 60 build/rect_probe $pt >> $O/rect.jsonl || exit 1
done
echo ok rect
timeout -k 10 300 python tools/tiles_ab.py --trials 2 --method cauchy_good --k 16 --m 4 --chunk 8388608 --json $O/tiles_cg164_8m.jsonl > $O/tiles.log 2>&1 &&
timeout -k 10 300 python tools/tiles_ab.py --trials 2 --method cauchy_good --k 20 --m 6 --chunk 8388608 --json $O/tiles_cg206_8m.jsonl >> $O/tiles.log 2>&1 && echo ok tiles
