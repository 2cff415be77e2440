# Stripe-server part size (column bytes per slot): 4 KiB (default) vs 8 / 16 KiB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/part_ab.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/part_ab_pytest.txt 2>&1 || { echo "small-call tests failed"; tail -20 gpurun_out/part_ab_pytest.txt; exit 1; }
for rep in 1 2; do
  for cfg in "16384 reed_sol_van" "65536 reed_sol_van" "16384 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128; do
      for kb in 4 8 16; do
        LSEC_SRV_PART_KB=$kb timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"part_kb\": $kb, \"rep\": $rep, /" >> $out || { echo "fail $kb $cfg T=$T"; exit 1; }
      done
    done
  done
done
echo "ok $(wc -l < $out)"
