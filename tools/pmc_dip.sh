#!/bin/bash
# The C = 8 MiB encode dip: counters of the c5 lows' encodes at C = 1 MiB and
# 8 MiB with equal bytes per launch -- Cauchy-good(20+6) and (16+4) (compiled packet networks,
# lsec_xornet) and RS(8+4) (k_gf8_bytewise).  One rocprofv3 --pmc pass per counter group and
# configuration, each with its own time limit; summary: tools/pmc_dip_summary.py gpurun_out/dip_<tag>.
#   gpurun -- bash tools/pmc_dip.sh <tag> [tcp sq ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-dip}
shift
out=gpurun_out/dip_${tag}
mkdir -p $out; export TMPDIR=/tmp
declare -A PASS
PASS[sq]="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAIT_ANY"
PASS[tcp]="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
PASS[lat]="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum"
CFGS=${DIP_CFGS:-"cauchy_good 20 6 1048576 1024|cauchy_good 20 6 8388608 128|cauchy_good 16 4 1048576 1024|cauchy_good 16 4 8388608 128|reed_sol_van 8 4 1048576 2048|reed_sol_van 8 4 8388608 256"}
passes=${*:-tcp sq}
IFS='|' read -ra CFGA <<< "$CFGS"
for pass in $passes; do
  P=${PASS[$pass]}
  for cfg in "${CFGA[@]}"; do
    set -- $cfg
    t="$1_k$2m$3c$(( $4 >> 20 ))"
    B0="python $PWD/bench.py --method $1 --k $2 --m $3 --chunk $4 --stripes $5 --steps 3 --warmup 1 --no-cpu --no-host-path --no-layout-ab --no-copy-ref --no-pmc"
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OLDPWD/$out/${t}_${pass}" -o p -- $B0) \
      > $out/${t}_${pass}.log 2>&1 || { echo "failed $t $pass"; tail -5 $out/${t}_${pass}.log; exit 1; }
    echo "ok $t $pass"
  done
done
