#!/bin/bash
# r04j: the remaining graph-mode mismatch (group 1's |STFT|^2 in two concurrent graphs): where the
# differing elements sit and what lies next to the buffer in device memory.
set -uo pipefail
O=gpurun_out/r04j
mkdir -p $O
DETAIL=1 timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 3 25 > $O/probe_detail.txt 2>&1; rc=$?
echo "rc $rc" >> $O/probe_detail.txt
grep -v "extent" $O/probe_detail.txt | head -60
exit $rc
