#!/bin/bash
# GPU box: host-path A/B of the in-place pinning threshold (tools/pin_run_ab.py), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/pin_run_ab.py > gpurun_out/pin_ab.jsonl 2> gpurun_out/pin_ab.err && echo pass1 && \
timeout -k 10 300 python -u tools/pin_run_ab.py --codes 6+3 --chunks 1048576,4194304 --reps 7 >> gpurun_out/pin_ab.jsonl 2>> gpurun_out/pin_ab.err && echo pass2
