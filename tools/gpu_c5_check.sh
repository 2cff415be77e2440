set -o pipefail
O=gpurun_out/c5chk; mkdir -p $O
for pt in "reed_sol_van 8+3 524288" "reed_sol_van 8+4 524288" "reed_sol_van 16+4 262144" "cauchy_good 16+4 262144" "cauchy_good 8+4 524288" "reed_sol_van 4+2 1048576" "reed_sol_van 6+3 1048576" "reed_sol_van 16+4 1048576"; do
  set -- $pt
  LSEC_TRACE=1 timeout -k 10 200 python tools/sweep.py --methods $1 --km $2 --chunks $3 --out $O/sweep.jsonl > /dev/null 2>> $O/trace.txt || exit 1
done
echo ok
