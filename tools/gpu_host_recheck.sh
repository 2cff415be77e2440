#!/bin/bash
# GPU box: one c5 point's host path measured again (tools/sweep.py, twice), e.g. a point that stood
# out in a full sweep.
#   gpurun -- bash tools/gpu_host_recheck.sh <tag> <method> <k+m> <chunk bytes>
set -o pipefail
tag=${1:-recheck}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
o=gpurun_out/host_recheck_${tag}.jsonl
: > $o
for i in 1 2; do
  timeout -k 10 240 python tools/sweep.py --methods $2 --km $3 --chunks $4 --out $o > /dev/null 2> gpurun_out/host_recheck_${tag}.err \
    || { echo "sweep failed"; tail -5 gpurun_out/host_recheck_${tag}.err; exit 1; }
done
python - "$o" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    if "method" in r:
        print(r["method"], r["k"], r["m"], r["chunk"], "dev enc", r["enc_hbm_frac"], "host enc / dec", r["host_enc_gibps"],
              r["host_dec_gibps"], "h2d link frac", r["enc_h2d_link_frac"])
PY
