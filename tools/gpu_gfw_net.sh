set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gfw_network or wide_fields" > gpurun_out/gfw_pytest.txt 2>&1 || { tail -30 gpurun_out/gfw_pytest.txt; exit 1; }
tail -2 gpurun_out/gfw_pytest.txt
for v in 0 0xff00 0x1000 0x4000; do
  LSEC_JIT_VARIANT=$v timeout -k 10 300 python tools/kbench.py --configs rs63w16,rs104w16,rs63w32,rs104w32,rs206w16 --variants "0,0;0,1" --rounds 3 > gpurun_out/gfw_kbench_$v.txt 2>&1 || { tail gpurun_out/gfw_kbench_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/gfw_kbench_$v.txt | grep -v amdgpu.ids
done
