#!/bin/bash
# GPU box, round 6: the free-after-op lifetime (verified per-stripe calls that free their buffers,
# the registration-window probe), the per-stripe fair table with the background unpinner off by
# default, the one-thread tail trace, and the decode's per-lane shapes.  Each step has its own limit.
#   gpurun --timeout 1200 -- bash tools/gpu_r06b.sh <tag> [free probe fair tail kdec]
set -o pipefail
tag=${1:-r06b}
shift
steps=${*:-free probe fair tail kdec}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp REF=oracle/_ref/libjerasure_ref.so
for s in $steps; do
  case $s in
    free)  # FNPTR_FREE_AFTER: every call's parity / stripe buffer malloc'd for it and freed after, each call verified
      o=gpurun_out/free_after_${tag}.jsonl; : > $o
      for c in "1048576 2 reed_sol_van encode 2" "1048576 4 reed_sol_van encode 2" "1048576 2 cauchy_good decode 2" \
               "1048576 4 cauchy_good decode 2" "1048576 3 cauchy_good decode 1" "4194304 2 reed_sol_van encode 1" \
               "4194304 3 cauchy_good decode 2" "2097152 2 reed_sol_van encode 2"; do
        set -- $c
        FNPTR_VERIFY=1 FNPTR_REF=$REF FNPTR_FREE_AFTER=$5 timeout -k 10 60 build/fnptr_bench $1 $2 2 $3 $4 >> $o \
          || { echo "free-after run failed: $c"; tail -3 $o; exit 1; }
      done
      python -c "
import json; rs=[json.loads(l) for l in open('$o')]
print('free-after verified calls', sum(r['verified'] for r in rs), 'mismatches', sum(r['mismatches'] for r in rs))" ;;
    churn)  # FNPTR_FREE_AFTER=2 (a fresh mmap per call): the engine's phases, the engine with no in-place
            # registration, and the reference, one thread and two
      o=gpurun_out/free_after_churn_${tag}.jsonl; : > $o
      for th in 1 2; do
        for e in "X=0" "LSEC_NO_HOST_REGISTER=1" "LSEC_OWN_DMA_MAX=0"; do
          env $e FNPTR_REF=$REF FNPTR_FREE_AFTER=2 timeout -k 10 60 build/fnptr_bench 1048576 $th 2 cauchy_good decode \
            | sed "s/}\$/, \"env\": \"$e\"}/" >> $o || { echo "churn run failed: $e"; exit 1; }
        done
      done
      LSEC_TRACE=1 FNPTR_FREE_AFTER=2 timeout -k 10 60 build/fnptr_bench 1048576 1 1 cauchy_good decode \
        > gpurun_out/free_after_churn_trace_${tag}.json 2> gpurun_out/free_after_churn_trace_${tag}.txt || { echo "traced churn failed"; exit 1; }
      python -c "
import json
for l in open('$o'):
    r = json.loads(l); print(r['impl'], r['threads'], r['env'], r['per_call_us_p50'], r['gibps'])"
      grep "lsec trace" gpurun_out/free_after_churn_trace_${tag}.txt | tail -3 ;;
    probe)
      timeout -k 10 240 python tools/probes/free_after_probe.py > gpurun_out/free_after_probe_${tag}.jsonl \
        || { echo "probe failed"; cat gpurun_out/free_after_probe_${tag}.jsonl; exit 1; }
      cat gpurun_out/free_after_probe_${tag}.jsonl ;;
    fair)
      timeout -k 10 600 bash tools/gpu_fnptr_fair.sh ${tag} 1048576:1:cauchy_good:decode 1048576:2:cauchy_good:decode \
        1048576:4:cauchy_good:decode 1048576:8:cauchy_good:decode 1048576:1:reed_sol_van:encode 1048576:2:reed_sol_van:encode \
        1048576:2:cauchy_good:decode:LSEC_DEFER_UNPIN_MB=256 1048576:2:cauchy_good:decode:FNPTR_FREE_AFTER=1 \
        1048576:2:reed_sol_van:encode:FNPTR_FREE_AFTER=1 65536:1:cauchy_good:decode 16384:1:cauchy_good:decode \
        > gpurun_out/fair_${tag}.log 2>&1 || { echo "fair failed"; tail -5 gpurun_out/fair_${tag}.log; exit 1; }
      python tools/fnptr_table.py gpurun_out/fnptr_fair_${tag}.jsonl ;;
    tail)
      timeout -k 10 200 bash tools/gpu_fnptr_tail.sh ${tag} || { echo "tail failed"; exit 1; } ;;
    kdec)  # decode per-lane shapes: 5,0 = shape 4 (8 B, the automatic one), 6,0 = 16 B, 7,0 = 32 B (branchy, R = 1 only)
      timeout -k 10 300 python tools/kbench.py --configs rs63,rs104,rs84c8 --variants "0,0;5,0;6,0;7,0" --rounds 5 \
        > gpurun_out/kdec_${tag}.txt 2>&1 || { echo "kbench failed"; tail -5 gpurun_out/kdec_${tag}.txt; exit 1; }
      grep variant gpurun_out/kdec_${tag}.txt ;;
  esac
done
