#!/bin/bash
# Strided DMA (issue_runs, ec_pinning.cpp): host-path parity tests, then the c5 host lows with
# strided copies off / on, and with in-place pinning at a lower run threshold.
set -o pipefail
O=gpurun_out/dma2d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "strided_dma or host_path or pinned or small_run or stripes_host or column_blocks" > $O/pytest.txt 2>&1 || { tail -5 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in "off LSEC_DMA_2D=0" "on LSEC_DMA_2D=1" "on_run6m LSEC_PIN_MIN_RUN_KB=6144"; do
  set -- $v
  for pt in "reed_sol_van 8+3 262144,524288,1048576" "reed_sol_van 8+4 524288" "reed_sol_van 4+2 1048576,8388608" "reed_sol_van 16+4 262144" "reed_sol_van 6+3 1048576" "reed_sol_van 20+6 4194304"; do
    set -- $1 $2 $pt
    env $2 timeout -k 10 200 python tools/sweep.py --dev-gib 0.25 --methods $3 --km $4 --chunks $5 --out $O/sweep_$1.jsonl > /dev/null 2>> $O/err.txt || exit 1
  done
  echo "ok $1"
done
