#!/bin/bash
# GPU box: one completion wait over all of a call's server parts (current build) vs one wait per
# part (build/oldlib), LStore's per-stripe encode_block pattern (tools/fnptr_bench.c), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/wait_all_ab.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wait_all_pytest.txt 2>&1 || { echo "small-call tests failed"; tail -20 gpurun_out/wait_all_pytest.txt; exit 1; }
echo "small-call tests ok: $(tail -1 gpurun_out/wait_all_pytest.txt)"
for rep in 1 2; do
  for cfg in "65536 reed_sol_van" "16384 reed_sol_van" "65536 cauchy_good" "16384 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128; do
      timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"build\": \"all\", \"rep\": $rep, /" >> $out || { echo "fail all $cfg T=$T"; exit 1; }
      LD_LIBRARY_PATH=$PWD/build/oldlib timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"build\": \"per-part\", \"rep\": $rep, /" >> $out || { echo "fail old $cfg T=$T"; exit 1; }
    done
  done
done
echo "ok $(wc -l < $out)"
