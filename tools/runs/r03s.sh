#!/bin/bash
# r03s: full GPU suite with the side-stream query branch (no record_stream); B = 1 timeline; C2 bench
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/bench_b1.json 2> $O/bench_b1.err
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1 -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/b1.out 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
echo done > $O/DONE
