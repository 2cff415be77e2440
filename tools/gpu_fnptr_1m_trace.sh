set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
export FNPTR_REF=oracle/_ref/libjerasure_ref.so
o=gpurun_out/fnptr_1m_s2d.jsonl
: > $o
for e in "X=1" "X=2" "LSEC_OWN_DMA_MAX=0" "X=3"; do
  env $e timeout -k 10 60 build/fnptr_bench 1048576 1 2 cauchy_good decode | sed "s/}\$/, \"env\": \"$e\"}/" >> $o || exit 1
done
LSEC_TRACE=1 FNPTR_ONLY_REF=0 timeout -k 10 60 build/fnptr_bench 1048576 1 1 cauchy_good decode > gpurun_out/trace_1m_s2d.json 2> gpurun_out/trace_1m_s2d.txt || exit 1
echo ok
