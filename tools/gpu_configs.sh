#!/bin/bash
# GPU-box: bench lines for the other BASELINE configs at N = 1 -- c4 (Cauchy-good 10+4, 4 MiB
# chunks) and c3's other lost shards (k-1, P0, P1 of RS 6+3) -- one process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --stripes 614 --steps 10 \
    --no-host-path >> gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit 1
for lost in 5 6 7; do
  timeout -k 10 300 python bench.py --lost $lost --steps 10 --no-cpu --no-host-path --no-layout-ab \
      >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.err || exit 1
done
echo done
