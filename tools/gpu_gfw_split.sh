#!/bin/bash
# w = 32 network shapes: for each LSEC_JIT_VARIANT, the network parity tests,
# then kbench on RS(10+4) / RS(6+3) at w = 32, then one SQ counter pass on RS(10+4).  Variant 0 is
# the default (the wave-pair slice split at 4 rows); 0x80000 the one-wave form.
#   gpurun -- bash tools/gpu_gfw_split.sh "0 0x80000"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/gfw; export TMPDIR=/tmp
variants=${1:-"0 0x80000"}
for v in $variants; do
  LSEC_JIT_VARIANT=$((v)) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k gfw_network -m gpu > gpurun_out/gfw/test_$v.log 2>&1 || { echo "tests failed $v"; tail -20 gpurun_out/gfw/test_$v.log; exit 1; }
  echo "tests ok $v"
done
for v in $variants; do
  LSEC_JIT_VARIANT=$((v)) timeout -k 10 300 python -u tools/kbench.py --configs rs104w32,rs63w32 --variants "0,0" --data-gib 8 --rounds 5 \
    > gpurun_out/gfw/kbench_$v.txt 2>&1 || { echo "kbench failed $v"; tail -20 gpurun_out/gfw/kbench_$v.txt; exit 1; }
  echo "== $v"; grep "N=" gpurun_out/gfw/kbench_$v.txt
done
P="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU"
for v in $variants; do
  (cd /tmp && LSEC_JIT_VARIANT=$((v)) timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OLDPWD/gpurun_out/gfw/pmc_$v" -o p -- \
    python $OLDPWD/tools/kbench.py --configs rs104w32 --variants "0,0" --data-gib 4 --rounds 1 --reps 2) > gpurun_out/gfw/pmc_$v.log 2>&1 \
    || { echo "pmc failed $v"; tail -5 gpurun_out/gfw/pmc_$v.log; exit 1; }
  echo "pmc ok $v"
done
