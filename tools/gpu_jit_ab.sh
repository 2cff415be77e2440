# A/B of XOR-network code shapes (LSEC_JIT_VARIANT) against the table kernel on wide RS codes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
OUT=gpurun_out/jit_ab.txt; : > $OUT
CFG=${CFG:-rs206,rs164,rs124}
LSEC_TRACE=1 timeout -k 10 200 python tools/kbench.py --configs $CFG --variants "2,0" --rounds 3 >> $OUT 2>&1 || exit 1
for v in ${VARIANTS:-0x41 0x43 0x1 0x3 0x0 0x2 0x10 0x12}; do
  echo "== LSEC_JIT_VARIANT=$v" >> $OUT
  LSEC_JIT_VARIANT=$((v)) LSEC_TRACE=1 timeout -k 10 200 python tools/kbench.py --configs $CFG --variants "0,0" --rounds 3 >> $OUT 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT
