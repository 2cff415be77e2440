#!/bin/bash
# After capping strided rows: host-path parity tests, c4 over 2 ranks on one GPU, and c5 points.
set -o pipefail
O=gpurun_out/d2c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "strided_dma or host_path or pinned or small_run or host_batches or column_blocks" > $O/pytest.txt 2>&1 || { tail -5 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --total-stripes 2048 --gpus 2 --share-gpus \
  --steps 5 --no-pmc --json-out $O/c4.json > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
for pt in "reed_sol_van 8+3 524288,2097152" "cauchy_good 10+4 4194304" "reed_sol_van 20+6 4194304"; do
  set -- $pt
  timeout -k 10 200 python tools/sweep.py --dev-gib 0.25 --methods $1 --km $2 --chunks $3 --out $O/sweep.jsonl > /dev/null 2>> $O/err.txt || exit 1
done
echo ok
