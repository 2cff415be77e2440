#!/bin/bash
# GPU box: longer verified stress of the per-stripe paths (tools/fnptr_bench.c FNPTR_VERIFY=1:
# every call's output overwritten before and compared with oracle/_ref after), 10 s per case; the
# 2-4 thread cases at 1-4 MiB run pinned in place; the last two free every call's buffer after it
# (FNPTR_FREE_AFTER: LStore's parity / stripe buffer lifetime; =2 a fresh mapping per call, so the
# in-place stall guard trips and the calls pack).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/stress_long.jsonl; : > $out
export FNPTR_VERIFY=1 FNPTR_REF=$PWD/oracle/_ref/libjerasure_ref.so
for cfg in "16384 256 reed_sol_van encode 0" "16384 256 cauchy_good decode 0" "65536 128 reed_sol_van encode 1" \
           "262144 64 cauchy_good encode 0" "1048576 48 reed_sol_van encode 0" "1048576 48 cauchy_good decode 0" \
           "1048576 2 cauchy_good decode 0" "1048576 3 reed_sol_van encode 0" "4194304 2 cauchy_good decode 0" \
           "4194304 4 reed_sol_van encode 0" "1048576 3 reed_sol_van encode 0 1" "1048576 2 cauchy_good decode 0 2"; do
  set -- $cfg
  FNPTR_FREE_AFTER=${6:-0} FNPTR_PINNED=$5 timeout -k 10 60 build/fnptr_bench $1 $2 10 $3 $4 >> $out || { echo "FAIL $cfg (rc $?)"; exit 1; }
done
python -c "
import json; rs=[json.loads(l) for l in open('$out')]
print('stress calls', sum(r['calls'] for r in rs), 'verified', sum(r['verified'] for r in rs), 'mismatches', sum(r['mismatches'] for r in rs))"
