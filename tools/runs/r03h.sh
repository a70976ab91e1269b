#!/bin/bash
# r03h: rows GEMM engine v2 (LDS epilogue tables, fragment prefetch): bitwise vs tiles, timings.
set -euo pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rows_engine" > $O/pytest_rows.log 2>&1
timeout -k 10 300 python tools/gemm_engines.py > $O/engines.txt 2>&1
echo done > $O/DONE
