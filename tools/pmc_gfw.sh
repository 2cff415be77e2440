#!/bin/bash
# GPU-box: PMC counters of the w = 16 / 32 RS kernels, the compiled network (variant 0,0) vs the
# generic transposed kernel (variant 0,1), each counter group in a pass of its own.
#   gpurun -- bash tools/pmc_gfw.sh <tag> [configs]
set -o pipefail
tag=${1:-gfw}
cfg=${2:-rs104w32,rs63w32}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "gpurun_out/pmc_${tag}_${name}" -o p -- \
    python tools/kbench.py --configs "$cfg" --variants "0,0;0,1" --rounds 1 --reps 2 --data-gib 8 \
    > "gpurun_out/pmc_${tag}_${name}.log" 2>&1 && echo "pass $name ok"
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run ic SQC_ICACHE_MISSES SQC_ICACHE_HITS ; \
run fetch FETCH_SIZE && run write WRITE_SIZE
