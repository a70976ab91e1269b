#!/bin/bash
# Row-kernel change check on the box: parity tests touching LN / dwconv, row-kernel timings, bench x2.
set -euo pipefail
TAG=${1:-rowops}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
timeout -k 10 120 python tools/rowops_bench.py > gpurun_out/$TAG/rowops.txt 2>/dev/null
for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.$r.json 2>/dev/null; done
