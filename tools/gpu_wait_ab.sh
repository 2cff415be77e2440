# Completion waits: parked waiters + poller (default) vs every waiter spinning (LSEC_WAIT=spin),
# LStore's per-stripe encode_block pattern, alternating, engine and reference legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/wait_ab.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_small_calls.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wait_ab_pytest.txt 2>&1 || { echo "small-call tests failed"; tail -20 gpurun_out/wait_ab_pytest.txt; exit 1; }
REF="$PWD/oracle/_ref/libjerasure_ref.so"
for rep in 1 2; do
  for cfg in "16384 reed_sol_van" "65536 reed_sol_van" "16384 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128; do
      for mode in park spin; do
        if [ $mode = spin ]; then export LSEC_WAIT=spin; else unset LSEC_WAIT; fi
        timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"wait\": \"$mode\", \"rep\": $rep, /" >> $out || { echo "fail $mode $cfg T=$T"; exit 1; }
      done
      unset LSEC_WAIT
      [ $rep = 1 ] && { FNPTR_REF=$REF timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | grep '"impl": "reference"' | sed "s/^{/{\"wait\": \"ref\", \"rep\": $rep, /" >> $out || true; }
    done
  done
done
echo "ok $(wc -l < $out)"
