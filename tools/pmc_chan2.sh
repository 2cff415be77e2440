#!/bin/bash
# Read requests per L2 channel (TCC instance 0-15, summed over the 8 XCDs; derived counters in
# tools/pmc_chan_counters.yaml) for an encode at C = 4 vs 8 MiB, same bytes per launch.
#   gpurun -- bash tools/pmc_chan2.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/chan2; export TMPDIR=/tmp
C=""; for n in $(seq 0 15); do C="$C LSEC_RDREQ_CH$n"; done
for cfg in "reed_sol_van 10 4 4194304 204" "reed_sol_van 10 4 8388608 102" "cauchy_good 12 4 4194304 170" "cauchy_good 12 4 8388608 85"; do
  set -- $cfg
  tag="$1_k$2m$3c$(( $4 >> 20 ))"
  B0="python $PWD/bench.py --method $1 --k $2 --m $3 --chunk $4 --stripes $5 --steps 2 --warmup 1 --no-cpu --no-host-path --no-layout-ab --no-copy-ref --no-pmc"
  (cd /tmp && timeout -s KILL 90 rocprofv3 -E "$OLDPWD/tools/pmc_chan_counters.yaml" --pmc $C --output-format csv -d "$OLDPWD/gpurun_out/chan2/$tag" -o p -- $B0) \
    > gpurun_out/chan2/$tag.log 2>&1 || { echo "failed $tag"; tail -5 gpurun_out/chan2/$tag.log; exit 1; }
  echo "ok $tag"
done
