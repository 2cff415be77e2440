# Completion-wait knobs: spinners allowed x spin duration, LStore's per-stripe encode_block pattern.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/wait_sweep.jsonl; : > $out
for rep in 1 2; do
  for cfg in "16384 reed_sol_van" "65536 reed_sol_van" "16384 cauchy_good"; do
    set -- $cfg
    for T in 1 8 32 128; do
      for knob in "8 100" "4 30" "2 20" "1 20" "0 0"; do
        set -- $cfg; n=${knob% *}; us=${knob#* }
        LSEC_WAIT_SPINNERS=$n LSEC_WAIT_SPIN_US=$us timeout -k 10 60 build/fnptr_bench $1 $T 2 $2 encode \
          | sed "s/^{/{\"spinners\": $n, \"spin_us\": $us, \"rep\": $rep, /" >> $out || { echo "fail $knob $cfg T=$T"; exit 1; }
      done
    done
  done
done
echo "ok $(wc -l < $out)"
