#!/bin/bash
# GPU box: what the slowest 1 % of one-thread 1 MiB decodes spend their time on.
# A traced run (LSEC_TRACE=2: per-call query / register / submit / drain / unpin; FNPTR_LAT_OUT: every
# call's latency) joined by tools/tail_join.py, then the untraced fair rows: the engine with the
# reference right after it in the same process, and the reference alone.
#   gpurun -- bash tools/gpu_fnptr_tail.sh <tag>
set -o pipefail
tag=${1:-tail}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export FNPTR_REF=oracle/_ref/libjerasure_ref.so
o=gpurun_out/fnptr_tail_${tag}
env -u FNPTR_REF LSEC_TRACE=2 FNPTR_LAT_OUT=$o.lat.txt timeout -k 10 90 build/fnptr_bench 1048576 1 5 cauchy_good decode \
  > $o.traced.jsonl 2> $o.trace.txt || { echo "traced run failed"; tail -5 $o.trace.txt; exit 1; }
python tools/tail_join.py $o.trace.txt $o.lat.txt > $o.join.jsonl || { echo "join failed"; exit 1; }
cat $o.join.jsonl
rm -f $o.trace.txt $o.lat.txt
: > $o.fair.jsonl
for rep in 1 2; do
  timeout -k 10 60 build/fnptr_bench 1048576 1 3 cauchy_good decode | sed "s/}\$/, \"env\": \"fair rep $rep\"}/" >> $o.fair.jsonl \
    || { echo "fair run failed"; exit 1; }
  FNPTR_ONLY_REF=1 timeout -k 10 60 build/fnptr_bench 1048576 1 3 cauchy_good decode | sed "s/}\$/, \"env\": \"reference alone rep $rep\"}/" >> $o.fair.jsonl \
    || { echo "reference run failed"; exit 1; }
done
cat $o.fair.jsonl
