#!/bin/bash
# Allocation A/B for the headline encode: per-XCD finish times of the
# encode's memory shape (tools/probes/xcd_balance.hip, static vs work-sharing tiles), and the
# engine's encode / decode over fresh allocations made by torch, hipMalloc and the VMM API in
# 2 MiB pieces (in order and shuffled) and 1 GiB pieces (tools/alloc_pmc_probe.py).
#   gpurun -- bash tools/gpu_alloc_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/alloc_ab; mkdir -p "$O"
timeout -k 10 300 python tools/probes/unregister_probe.py > "$O/unregister_probe.jsonl" 2> "$O/unregister_probe.err" || echo "unregister probe failed"
timeout -k 10 240 build/xcd_balance 8 4096 > "$O/xcd_balance.jsonl" 2>&1 || { echo "xcd_balance failed"; tail -3 "$O/xcd_balance.jsonl"; exit 1; }
echo "ok xcd_balance"
timeout -k 10 600 python tools/alloc_pmc_probe.py --trials 15 --alloc torch,hipmalloc,vmm:2,vmm:2:shuffle,vmm:1024 \
  --json "$O/alloc_kinds.jsonl" > "$O/alloc_kinds.log" 2>&1 || { echo "alloc kinds failed"; tail -5 "$O/alloc_kinds.log"; exit 1; }
echo "ok alloc kinds"
