#!/bin/bash
# Scan change check on the box: scan parity tests, scan alone at 16/32 clips, bench x2.
set -euo pipefail
TAG=${1:-scan}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_scan_fma.py tests/test_gpu_parity.py -k "scan or fma" -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
for m in 2 0; do for b in 16 32; do timeout -k 10 60 python tools/scan_bench.py $b 501 384 64 $m 100 2>/dev/null >> gpurun_out/$TAG/scan.txt; done; done
for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.$r.json 2>/dev/null; done
