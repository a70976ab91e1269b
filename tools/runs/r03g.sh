#!/bin/bash
# r03g: rows GEMM engine: bitwise vs tiles, isolated timings, bench A/B.
set -euo pipefail
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rows_engine" > $O/pytest_rows.log 2>&1
timeout -k 10 300 python tools/gemm_engines.py > $O/engines.txt 2>&1
timeout -k 10 900 python tools/ab_matrix.py $O/ab 2 'tiles|VASR_GEMM_ENGINE=1|' 'rows|VASR_GEMM_ENGINE=2|' > $O/ab.out 2>&1
echo done > $O/DONE
