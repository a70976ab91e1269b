#!/bin/bash
# r03c: scan split into per-N objects + N = 128 + padded state dims: scan/state-dim/ragged GPU tests,
# then the whole GPU suite, then the default bench.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "state_dim or n128 or zero_framed or scan" > $O/pytest_focus.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
for N in 16 32 64 128; do timeout -k 10 60 python tools/scan_bench.py 16 501 384 $N 2 50 >> $O/scan_bench.txt 2>&1; done
echo done > $O/DONE
