#!/bin/bash
# Host-path call patterns (tools/probes/host_pattern.py) with and without the sweep's device phase,
# and with the device staging budget at its default and at the packed budget.
set -o pipefail
O=gpurun_out/hostpat; mkdir -p $O
P="timeout -k 10 120 python tools/probes/host_pattern.py --km 8+3 --chunk 524288 --pattern EEEDDDEDEDED"
LSEC_TRACE=1 $P --tag default >> $O/pattern.jsonl 2>> $O/trace.txt &&
LSEC_TRACE=1 $P --tag default --dev-first >> $O/pattern.jsonl 2>> $O/trace.txt &&
LSEC_TRACE=1 LSEC_DEV_STAGING_MB=128 $P --tag dev128 --dev-first >> $O/pattern.jsonl 2>> $O/trace.txt &&
echo ok
