#!/bin/bash
# Host-path call patterns (tools/probes/host_pattern.py) after the sweep's device phase: freed to
# the driver at once, freed then a pause, kept in torch's cache.
set -o pipefail
O=gpurun_out/hostpat2; mkdir -p $O
P="timeout -k 10 120 python tools/probes/host_pattern.py --km 8+3 --chunk 524288 --pattern EDEDEDEEE --dev-first"
LSEC_TRACE=1 $P --tag freed >> $O/pattern.jsonl 2>> $O/trace.txt &&
LSEC_TRACE=1 $P --tag sleep2 --sleep 2 >> $O/pattern.jsonl 2>> $O/trace.txt &&
LSEC_TRACE=1 $P --tag cached --keep-cache >> $O/pattern.jsonl 2>> $O/trace.txt &&
echo ok
