#!/bin/bash
# Issue side of the C = 4 vs 8 MiB encode dip: SQ counters of RS(10+4) and
# Cauchy-good(12+4) encodes at the same bytes per launch, C = 4 MiB and 8 MiB, plus the decodes.
# One pass of eight SQ counters, with the kernel trace for durations (pmc_dram.sh covers the memory
# side).  Summaries: tools/pmc_sq_summary.py gpurun_out/sq.
#   gpurun -- bash tools/pmc_sq.sh [sq tcp1 tcp2]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/sq; export TMPDIR=/tmp
# passes (each its own run): sq = issue side; tcp1 / tcp2 = the vector L1 / address path between
# the SQ and the L2 (stalls, L1 -> L2 read latency, translation misses and stalls)
declare -A PASS
PASS[sq]="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAIT_ANY"
PASS[tcp1]="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
PASS[tcp2]="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum"
passes=${*:-sq}
for pass in $passes; do
P=${PASS[$pass]}
for cfg in "reed_sol_van 10 4 4194304 204" "reed_sol_van 10 4 8388608 102" "cauchy_good 12 4 4194304 170" "cauchy_good 12 4 8388608 85"; do
  set -- $cfg
  tag="$1_k$2m$3c$(( $4 >> 20 ))"
  B0="python $PWD/bench.py --method $1 --k $2 --m $3 --chunk $4 --stripes $5 --steps 3 --warmup 1 --no-cpu --no-host-path --no-layout-ab --no-copy-ref --no-pmc"
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OLDPWD/gpurun_out/sq/${tag}_${pass}" -o p -- $B0) \
    > gpurun_out/sq/${tag}_${pass}.log 2>&1 || { echo "failed $tag"; tail -5 gpurun_out/sq/${tag}_${pass}.log; exit 1; }
  echo "ok $tag"
done
done
