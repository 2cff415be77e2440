#!/bin/bash
# c4 (Cauchy-good(10+4), 4 MiB) over 2 ranks on the box's one GPU: host path with strided copies
# on and off, alternating.
set -o pipefail
O=gpurun_out/c4ab; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in "on X=1" "off LSEC_DMA_2D=0"; do
    set -- $v
    env $2 timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --total-stripes 2048 --gpus 2 --share-gpus \
      --steps 5 --no-pmc --json-out $O/c4_$1_$r.json > $O/c4_$1_$r.log 2>&1 || { tail -5 $O/c4_$1_$r.log; exit 1; }
  done
  echo "ok $r"
done
