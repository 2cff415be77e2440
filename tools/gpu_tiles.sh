#!/bin/bash
# Work-sharing tiles on the box: the A/B on the headline (tools/tiles_ab.py), then the bench line
# under rocprofv3 --kernel-trace --stats and a plain bench run.   gpurun -- bash tools/gpu_tiles.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-t}; O=gpurun_out/tiles_$tag; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 python tools/tiles_ab.py --trials 4 --json "$O/tiles_ab.jsonl" > "$O/tiles_ab.log" 2>&1 || { echo "tiles_ab failed"; tail -5 "$O/tiles_ab.log"; exit 1; }
echo "ok tiles_ab"; cat "$O/tiles_ab.jsonl"
