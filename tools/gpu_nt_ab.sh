#!/bin/bash
# GPU box: host-path rates with streaming-store host copies (default) vs plain memcpy
# (LSEC_NT_COPY=0), alternating processes: the c5 host path at small chunks (packed) and 1 MiB
# per-stripe calls.   gpurun -- bash tools/gpu_nt_ab.sh <tag>
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for nt in 1 0; do
    LSEC_NT_COPY=$nt timeout -k 10 300 python tools/sweep.py --methods reed_sol_van --km 8+4,6+3 --chunks 262144,524288 \
      --dev-gib 1 --out "gpurun_out/nt_ab_${tag}_r${round}_nt${nt}.jsonl" > "gpurun_out/nt_ab_${tag}.log" 2>&1 \
      || { echo "sweep failed"; tail -20 "gpurun_out/nt_ab_${tag}.log"; exit 1; }
    python - "gpurun_out/nt_ab_${tag}_r${round}_nt${nt}.jsonl" "$round" "$nt" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f"round {sys.argv[2]} nt {sys.argv[3]}: RS({r['k']}+{r['m']}) C={r['chunk'] >> 10} KiB host enc {r['host_enc_gibps']:.1f} dec {r['host_dec_gibps']:.1f} GiB/s exact {r['bit_exact']}")
PY
  done
done
