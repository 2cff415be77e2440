#!/bin/bash
# Config c1 (segment write / read / inspect) under the host-path knobs of round 5: default, the
# round-4 in-place run threshold, strided copies off.  Alternating, twice.
set -o pipefail
O=gpurun_out/c1ab; mkdir -p $O
for r in 1 2; do
  for v in "default X=1" "run2560 LSEC_PIN_MIN_RUN_KB=2560" "no2d LSEC_DMA_2D=0"; do
    set -- $v
    env $2 timeout -k 10 300 python -u tools/c1_depot.py > $O/c1_$1_$r.log 2>&1 || { tail -5 $O/c1_$1_$r.log; exit 1; }
  done
  echo "ok $r"
done
