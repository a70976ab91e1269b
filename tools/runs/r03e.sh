#!/bin/bash
# r03e: B = 1 timelines (10 s, 30 s) inside the graph, and the B = 1 latency bench lines.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1_10s -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/b1_10s.out 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1_30s -o run --output-format csv -- python3 tools/graph_copies.py 1 480000 1 > $O/b1_30s.out 2>&1
timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/b1_10s.json 2> $O/b1_10s.err
echo done > $O/DONE
