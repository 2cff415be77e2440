#!/bin/bash
# Per-stripe 1 MiB Cauchy-good(6+3) decodes at two threads: LSEC_TRACE phases per call, and a
# kernel + memory-copy timeline under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/t2; mkdir -p $O
export FNPTR_REF=$GRAFT_REPO_ROOT/oracle/_ref/libjerasure_ref.so TMPDIR=/tmp
[ -n "$SKIP_TRACE" ] || LSEC_TRACE=1 timeout -k 10 60 build/fnptr_bench 1048576 2 1 cauchy_good decode > $O/trace.json 2> $O/trace.txt || exit 1
echo ok trace
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
   $GRAFT_REPO_ROOT/build/fnptr_bench 1048576 2 1 cauchy_good decode) > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo ok prof
