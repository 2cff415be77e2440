#!/bin/bash
# A/B of the fn-pointer call pattern: current library vs build/oldlib (LD_LIBRARY_PATH), and
# the current library with LSEC_NO_PINNED_DMA=1.  Interleaved, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/fnptr_ab.txt
for rep in 1 2; do
for cfg in "16384 1 48" "16384 128 48" "1048576 1 16" "1048576 32 16"; do
  set -- $cfg
  echo "cur  $cfg $(timeout -k 10 120 ./build/fnptr_bench $1 $2 $3 cauchy_good 2>&1 | grep chunk)" >> $out || exit 1
  echo "nopin $cfg $(LSEC_NO_PINNED_DMA=1 timeout -k 10 120 ./build/fnptr_bench $1 $2 $3 cauchy_good 2>&1 | grep chunk)" >> $out || exit 1
  echo "old  $cfg $(LD_LIBRARY_PATH=$PWD/build/oldlib timeout -k 10 120 ./build/fnptr_bench $1 $2 $3 cauchy_good 2>&1 | grep chunk)" >> $out || exit 1
done
done
echo done
