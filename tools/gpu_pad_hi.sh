#!/bin/bash
# GPU box: the C = 8 MiB encode dip against large shard pads (tools/kbench.py --pad: bytes after
# every shard row).  Round 4's pads (256 B - 68 KiB) left it as it was; pads of 256 KiB - 3 MiB move the
# shards' address bits 18-23 apart, which tells whether the dip is the K + R streams of a stripe
# sharing their high address bits (shards 8 MiB apart differ only from bit 23 up).
#   gpurun -- bash tools/gpu_pad_hi.sh <tag>
set -o pipefail
tag=${1:-pad}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/pad_hi_${tag}.txt
: > $o
for pad in 0 262144 1048576 3145728 0; do
  echo "== pad $pad" >> $o
  timeout -k 10 240 python tools/kbench.py --configs rs84,rs84c8,cg164c8,cg206c8 --variants "0,0" --rounds 3 --data-gib 16 --pad $pad \
    >> $o 2>&1 || { echo "kbench failed at pad $pad"; tail -5 $o; exit 1; }
done
grep -E "==|variant" $o
