#!/bin/bash
# GPU box: host-path A/B of the in-place pinning threshold at small chunks (tools/pin_run_ab.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/pin_run_ab.py --chunks 16384,65536,131072 --gib 0.5 > gpurun_out/pin_ab2.jsonl 2> gpurun_out/pin_ab2.err && echo pass1 && \
timeout -k 10 400 python -u tools/pin_run_ab.py --codes 6+3 --chunks 65536,262144 --gib 0.1 --reps 9 >> gpurun_out/pin_ab2.jsonl 2>> gpurun_out/pin_ab2.err && echo pass2
