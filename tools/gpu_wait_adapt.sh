# Adaptive spinning on / off (LSEC_WAIT_ADAPT), alternating in one process sequence per config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/wait_adapt.jsonl; : > $out
for rep in 1 2 3; do
  for cfg in "16384 reed_sol_van" "16384 cauchy_good" "65536 reed_sol_van"; do
    set -- $cfg
    for T in 1 8 32 128; do
      for ad in 1 0; do
        LSEC_WAIT_ADAPT=$ad timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode | sed "s/^{/{\"adapt\": $ad, \"rep\": $rep, /" >> $out || { echo "fail"; exit 1; }
      done
    done
  done
done
echo "ok $(wc -l < $out)"
