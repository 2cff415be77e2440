#!/bin/bash
# c4's host shape (Cauchy-good(10+4), 4 MiB, ~2.9 GiB per call) in one process, strided copies on /
# off; then the 2-rank rehearsal with per-call phases (LSEC_TRACE) for both.
set -o pipefail
O=gpurun_out/c4ab2; mkdir -p $O; export TMPDIR=/tmp
for v in "on X=1" "off LSEC_DMA_2D=0"; do
  set -- $v
  env $2 timeout -k 10 200 python tools/sweep.py --dev-gib 0.25 --host-gib 2.85 --methods cauchy_good --km 10+4 --chunks 4194304 \
    --out $O/sweep_$1.jsonl > /dev/null 2>> $O/err.txt || exit 1
done
echo ok sweep
for v in "on X=1" "off LSEC_DMA_2D=0"; do
  set -- $v
  env $2 LSEC_TRACE=1 timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --total-stripes 2048 --gpus 2 --share-gpus \
    --steps 5 --no-pmc --json-out $O/c4_$1.json > $O/c4_$1.log 2>&1 || { tail -5 $O/c4_$1.log; exit 1; }
done
echo ok ranks
