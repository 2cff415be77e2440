#!/bin/bash
# Host path A/B: pageable buffers pinned in place (default) vs packed (LSEC_NO_HOST_REGISTER=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
  for mode in reg noreg; do
    if [ $mode = noreg ]; then export LSEC_NO_HOST_REGISTER=1; else unset LSEC_NO_HOST_REGISTER; fi
    timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-layout-ab --stripes 512 > gpurun_out/hr_$mode.log 2>&1 || exit 1
    echo "$mode $(grep '^{"metric"' gpurun_out/hr_$mode.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["host_path"]; print(d["encode_gibps"], d["decode_gibps"], d["pinned"]["encode_gibps"], d["pinned"]["decode_gibps"])')" >> gpurun_out/hostreg_ab.txt
  done
done
echo done
