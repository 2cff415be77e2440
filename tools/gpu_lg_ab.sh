#!/bin/bash
# GPU box: bytewise encode with all input loads in flight (variant 0,0) vs loads two shards at
# a time (6,0 -> shape 5, LG = 2), LStore's unpadded layout and a 1 KiB pad, with the XOR mix
# probe beside them (tools/kbench.py, interleaved rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kbench.py --configs rs63,rs104,rs84 --variants "0,0;6,0" --mix > gpurun_out/lg_ab_pad0.txt 2>&1 || { tail -5 gpurun_out/lg_ab_pad0.txt; exit 1; }
echo pad0 ok
timeout -k 10 300 python -u tools/kbench.py --configs rs63 --variants "0,0;6,0" --mix --pad 1024 > gpurun_out/lg_ab_pad1k.txt 2>&1 || { tail -5 gpurun_out/lg_ab_pad1k.txt; exit 1; }
echo pad1k ok
