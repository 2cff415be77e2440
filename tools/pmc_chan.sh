#!/bin/bash
# Per-L2-channel memory requests (TCC_EA0_RDREQ / WRREQ without _sum: one value per TCC instance)
# for an encode at C = 4 vs 8 MiB with the same bytes per launch: is the 8 MiB dip a channel
# imbalance?  One rocprofv3 --pmc pass per counter.   gpurun -- bash tools/pmc_chan.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/chan; export TMPDIR=/tmp
for cfg in "reed_sol_van 10 4 4194304 204" "reed_sol_van 10 4 8388608 102" "cauchy_good 12 4 4194304 170" "cauchy_good 12 4 8388608 85"; do
  set -- $cfg
  tag="$1_k$2m$3c$(( $4 >> 20 ))"
  B0="python $PWD/bench.py --method $1 --k $2 --m $3 --chunk $4 --stripes $5 --steps 3 --warmup 1 --no-cpu --no-host-path --no-layout-ab --no-copy-ref --no-pmc"
  timeout -k 10 120 $B0 --json-out gpurun_out/chan/bench_$tag.json > gpurun_out/chan/bench_$tag.log 2>&1 || exit 1
  for c in TCC_EA0_RDREQ TCC_EA0_WRREQ; do
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$OLDPWD/gpurun_out/chan/${c}_$tag" -o p -- $B0) \
      > gpurun_out/chan/${c}_$tag.log 2>&1 || exit 1
  done
  echo "ok $tag"
done
