# Stripe-server workgroup count A/B: 32 (the in-tree build) vs 64 / 128 (build/srv<N>), LStore's
# per-stripe encode_block pattern, engine only, pageable buffers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/srv_wg.jsonl; : > $out
for rep in 1 2; do
for wg in 32 64 128; do
  bin=build/fnptr_bench; [ $wg != 32 ] && bin=build/srv$wg/build/fnptr_bench
  for cfg in "16384 reed_sol_van" "65536 reed_sol_van" "16384 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128; do
      timeout -k 10 60 $bin $1 $T 2 $2 encode | sed "s/^{/{\"srv_wg\": $wg, \"rep\": $rep, /" >> $out || { echo "fail wg=$wg $cfg T=$T"; exit 1; }
    done
  done
done
done
echo "ok $(wc -l < $out)"
