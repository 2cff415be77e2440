#!/bin/bash
# Allocation placement modes of the headline encode: fresh allocations in one
# process, timed, then one rocprofv3 --pmc pass per counter group over the same probe (each pass its
# own process, so its own allocations; tools/alloc_pmc_summary.py correlates counters with launch
# time across the trials of each pass).
#   gpurun -- bash tools/gpu_alloc_modes.sh [list] [time] [pass ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
O=$R/gpurun_out/alloc; mkdir -p "$O"; export TMPDIR=/tmp
declare -A PASS
PASS[tcp1]="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
PASS[tcp2]="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum"
PASS[dram1]="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
PASS[dram2]="TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum"
PASS[chan]="$(for n in $(seq 0 15); do printf 'LSEC_RDREQ_CH%d ' $n; done)"
PASS[wchan]="$(for n in $(seq 0 15); do printf 'LSEC_WRREQ_CH%d ' $n; done)"
PASS[xcc]="$(for n in $(seq 0 7); do printf 'LSEC_RDREQ_XCC%d LSEC_RDLEV_XCC%d ' $n $n; done)"
PASS[xcc2]="$(for n in $(seq 0 7); do printf 'LSEC_RDCS_XCC%d LSEC_RDGMI_XCC%d ' $n $n; done)"
PASS[gmi]="TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_IO_32B_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum"
PASS[wgmi]="TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum"
PASS[utcl]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
PASS[extra]="${LSEC_EXTRA_PMC:-}"
TRIALS=${TRIALS:-8}
PROBE="python $R/tools/alloc_pmc_probe.py --trials $TRIALS ${PROBE_ARGS:-}"
steps=${*:-list time}
for step in $steps; do
  case $step in
  list)
    (cd /tmp && timeout -s KILL 60 rocprofv3 -L) > "$O/avail.txt" 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
    echo "ok list" ;;
  time)
    timeout -k 10 300 $PROBE --json "$O/time.jsonl" > "$O/time.log" 2>&1 || { echo "time failed"; tail -5 "$O/time.log"; exit 1; }
    echo "ok time" ;;
  *)
    P=${PASS[$step]}
    [ -n "$P" ] || { echo "unknown pass $step"; exit 1; }
    mkdir -p "$O/$step"
    (cd /tmp && timeout -s KILL 180 rocprofv3 -E "$R/tools/pmc_alloc_counters.yaml" \
        --pmc $P --output-format csv -d "$O/$step" -o p -- $PROBE --json "$O/$step/trials.jsonl") \
      > "$O/$step.log" 2>&1 || { echo "failed $step"; tail -5 "$O/$step.log"; exit 1; }
    echo "ok $step" ;;
  esac
done
