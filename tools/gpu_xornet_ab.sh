#!/bin/bash
# A/B of w = 8 XOR-network (K1b) variants on wide RS codes, interleaved on one box, after the
# parity cases.  Usage: tools/gpu_xornet_ab.sh <tag> <variant> [...]
# (the first variant is the baseline; LSEC_JIT_VARIANT bits, see ec_jit.cpp); CFGS="config:lost ..." overrides
# the codes timed; the parity cases run under the default variant
set -o pipefail
tag=$1; shift
out=gpurun_out/xab_$tag
mkdir -p $out
LSEC_JIT_VARIANT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "xor_network or wide_stripes or gfw_network or bitmatrix_network" > $out/pytest.txt 2>&1 \
  || { echo "parity failed"; tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for round in 1 2; do
  for v in "$@"; do
    for cfg in ${CFGS:-rs248:0,1,2,3,4,5,6,7 rs206:0,1,2,3,4,5 rs206:0 rs128:0,1,2,3,4,5,6,7}; do
      c=${cfg%%:*} lost=${cfg#*:}
      LSEC_JIT_VARIANT=$((v)) timeout -k 10 240 python -u tools/kbench.py --configs $c --lost $lost --variants "0,0" \
        --data-gib 8 --rounds 3 > $out/k.txt 2>&1 || { echo "kbench failed $v $cfg"; tail -20 $out/k.txt; exit 1; }
      echo "r${round}_${c}_${lost}_v${v}: $(grep 'N=' $out/k.txt | tail -1)"
    done
  done
done
