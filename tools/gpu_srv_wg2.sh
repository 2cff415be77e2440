# Stripe server: workgroups 32 / 64 / 128 with pageable and page-locked callers (page-locked
# callers leave the host CPUs idle, so their rate is the server's own), after the wait changes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/srv_wg2.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/srv_wg2_pytest.txt 2>&1 || { echo "small-call tests failed"; tail -20 gpurun_out/srv_wg2_pytest.txt; exit 1; }
for wg in 32 64 128; do
  bin=build/fnptr_bench; [ $wg != 32 ] && bin=build/srv$wg/build/fnptr_bench
  for cfg in "16384 reed_sol_van" "16384 cauchy_good" "65536 reed_sol_van"; do
    set -- $cfg
    for T in 1 8 32 128; do
      for pin in 0 1; do
        FNPTR_PINNED=$pin timeout -k 10 60 $bin $1 $T 2 $2 encode | sed "s/^{/{\"srv_wg\": $wg, /" >> $out || { echo "fail wg=$wg $cfg T=$T"; exit 1; }
      done
    done
  done
done
echo "ok $(wc -l < $out)"
