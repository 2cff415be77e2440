#!/bin/bash
# Strided copies under rocprofv3 (SDMA or blit kernel?) and with two processes at once.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/rect2; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- \
   $GRAFT_REPO_ROOT/build/rect_probe 10 4 4194304 36) > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo ok prof
timeout -k 10 120 build/rect_probe 10 4 4194304 36 > $O/single.jsonl || exit 1
timeout -k 10 120 build/rect_probe 10 4 4194304 36 > $O/pair_a.jsonl & pa=$!
timeout -k 10 120 build/rect_probe 10 4 4194304 36 > $O/pair_b.jsonl & pb=$!
wait $pa || exit 1
wait $pb || exit 1
echo ok pair
