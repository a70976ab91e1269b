#!/bin/bash
# r04i: graph-captured interference (real overlap): which concurrently running kernel changes the
# |STFT|^2 output (the remaining graph-mode mismatch after the scan fix), and the scan re-checked.
set -uo pipefail
O=gpurun_out/r04i
mkdir -p $O
VICTIMS="stft;scan" timeout -k 10 400 python -u tools/diag/interference_graph.py 20 3 > $O/igraph.txt 2>&1; rc=$?
echo "rc $rc" >> $O/igraph.txt
grep -v libdrm $O/igraph.txt | awk '$0 !~ / 0\/60/' | head -80
exit $rc
