#!/bin/bash
# r03o: per-kernel census of the bench step (32 x 10 s, two 16-clip groups) after the rows engine / tail forms
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b32 -o run --output-format csv -- python3 tools/graph_copies.py 32 160000 2 > $O/b32.out 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1_30 -o run --output-format csv -- python3 tools/graph_copies.py 1 480000 1 > $O/b1_30.out 2>&1
echo done > $O/DONE
