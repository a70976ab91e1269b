#!/bin/bash
# r03an: concurrent two-group graph replay mismatch -- bisect (streaming vs chunked scan), the chained
# replay of small groups (GraphedTranscriber.serial), and the bench's 16-clip groups.
set -uo pipefail
O=gpurun_out/r03an
mkdir -p $O
VASR_SCAN_CHUNKED=0 timeout -k 10 250 python tools/diag/graph_stress.py own 2 > $O/own2_streaming.txt 2>&1
VASR_SCAN_CHUNKED=1 timeout -k 10 250 python tools/diag/graph_stress.py own 2 > $O/own2_chunked.txt 2>&1
timeout -k 10 250 python tools/diag/graph_stress.py caller 2 > $O/caller2_serial.txt 2>&1
timeout -k 10 250 python tools/diag/graph_stress.py caller 32 > $O/caller32.txt 2>&1
timeout -k 10 100 python tools/diag/graph_caches.py > $O/caches.txt 2>&1
grep -h MODE $O/*.txt; cat $O/caches.txt
