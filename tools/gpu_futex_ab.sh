#!/bin/bash
# GPU box: lock-free futex parking with a multi-flag wait per call (current build) vs HEAD's
# mutex + condition-variable parking with one wait per part (build/oldlib), LStore's per-stripe
# encode_block pattern (tools/fnptr_bench.c), alternating; LSEC_STATS route counters on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/futex_ab.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/futex_pytest.txt 2>&1 || { echo "tests failed"; tail -20 gpurun_out/futex_pytest.txt; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/futex_pytest.txt)"
for rep in 1 2; do
  for cfg in "16384 reed_sol_van" "65536 reed_sol_van" "16384 cauchy_good" "65536 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128 256; do
      LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode 2>gpurun_out/futex_stats.txt | sed "s/^{/{\"build\": \"futex\", \"rep\": $rep, /" >> $out || { echo "fail new $cfg T=$T"; exit 1; }
      echo "$1 $2 T=$T $(cat gpurun_out/futex_stats.txt)" >> gpurun_out/futex_routes.txt
      LD_LIBRARY_PATH=$PWD/build/oldlib timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"build\": \"head\", \"rep\": $rep, /" >> $out || { echo "fail old $cfg T=$T"; exit 1; }
    done
  done
done
echo "ok $(wc -l < $out)"
