#!/bin/bash
# Fresh allocations of the headline workload by torch, hipMalloc and the VMM API (2 MiB pieces in
# order and shuffled, 1 GiB pieces), engine encode / decode on each (tools/alloc_pmc_probe.py);
# and whether PCIe carries both directions at once (tools/probes/duplex_probe.cpp).
#   gpurun -- bash tools/gpu_alloc_kinds.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/alloc_kinds_${1:-a}; mkdir -p "$O"
timeout -k 10 120 build/duplex_probe 512 > "$O/duplex.jsonl" 2>&1 || { echo "duplex failed"; cat "$O/duplex.jsonl"; exit 1; }
cat "$O/duplex.jsonl"
timeout -k 10 900 python tools/alloc_pmc_probe.py --trials 15 --alloc torch,vmm:2:shuffle,vmm:2,hipmalloc,vmm:1024 \
  --json "$O/alloc_kinds.jsonl" > "$O/alloc_kinds.log" 2>&1 || { echo "alloc kinds failed"; tail -5 "$O/alloc_kinds.log"; exit 1; }
echo "ok alloc kinds"
