#!/bin/bash
# Memory-side queueing at C = 4 vs 8 MiB (same bytes per launch): outstanding-request levels
# (average latency = LEVEL / REQ in cycles), DRAM credit stalls and write stalls.  Two passes of
# four TCC counters each, with the kernel trace for durations.   gpurun -- bash tools/pmc_dram.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/dram; export TMPDIR=/tmp
P1="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
P2="TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum"
for cfg in "reed_sol_van 10 4 4194304 204" "reed_sol_van 10 4 8388608 102" "cauchy_good 12 4 4194304 170" "cauchy_good 12 4 8388608 85"; do
  set -- $cfg
  tag="$1_k$2m$3c$(( $4 >> 20 ))"
  B0="python $PWD/bench.py --method $1 --k $2 --m $3 --chunk $4 --stripes $5 --steps 2 --warmup 1 --no-cpu --no-host-path --no-layout-ab --no-copy-ref --no-pmc"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OLDPWD/gpurun_out/dram/${tag}_p$i" -o p -- $B0) \
      > gpurun_out/dram/${tag}_p$i.log 2>&1 || { echo "failed $tag p$i"; tail -5 gpurun_out/dram/${tag}_p$i.log; exit 1; }
  done
  echo "ok $tag"
done
