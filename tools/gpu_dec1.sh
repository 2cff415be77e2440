set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "X=0" "LSEC_HOST_BLOCKS=1" "LSEC_PIN_MIN_RUN_KB=1024" "LSEC_PIN_MIN_RUN_KB=1024 LSEC_KERNEL_COPY=1" "LSEC_HOST_BLOCKS=3"; do
  env $v FNPTR_SET_MB=2048 timeout -k 10 60 build/fnptr_bench 1048576 1 2 cauchy_good decode | sed "s/}\$/, \"env\": \"$v\"}/" >> gpurun_out/dec1.jsonl || exit 1
  env $v LSEC_TRACE=1 FNPTR_SET_MB=2048 timeout -k 10 60 build/fnptr_bench 1048576 1 0.3 cauchy_good decode 2> gpurun_out/dec1_trace_$(echo $v | tr ' =' '__').txt > /dev/null || exit 1
done
