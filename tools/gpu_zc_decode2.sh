#!/bin/bash
# GPU box: pageable 16 KiB Cauchy-good(6+3) decode_block at 128 threads under wait-knob variants
# (LSEC_STATS=1), to find what spends the CPU quota (tools/fnptr_bench.c).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/zc_decode2.txt; : > $out
run() {
  echo "== $*" >> $out
  env "$@" LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 128 2 cauchy_good decode >> $out 2>&1 || { echo "fail $*"; exit 1; }
}
run X=default
run LSEC_WAIT_SPINNERS=0
run LSEC_WAIT_ADAPT=0 LSEC_WAIT_SPINNERS=0
run LSEC_WAIT_POLLERS=1
run LSEC_PTR_CHECK=first
run X=default
echo "== encode default" >> $out
LSEC_STATS=1 timeout -k 10 60 build/fnptr_bench 16384 128 2 cauchy_good encode >> $out 2>&1 || exit 1
echo ok
