#!/bin/bash
# Fused-tail rows per workgroup (VASR_TAIL_ROWS=16|32): tail parity tests with the 16-row form,
# the isolated tail over M, and interleaved bench lines (C2 fp32, C3 bf16).
set -euo pipefail
OUT=gpurun_out/tailrows; mkdir -p $OUT
VASR_TAIL_ROWS=16 timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest16.log 2>&1
for r in 32 16; do VASR_TAIL_ROWS=$r timeout -k 10 120 python tools/tail_bench.py 501 1024 8016 16032 > $OUT/tail_$r.txt 2>&1; done
for i in 1 2; do for r in 32 16; do
  VASR_TAIL_ROWS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/bench_c2_$r.$i.json 2>/dev/null
  VASR_TAIL_ROWS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter --bf16 > $OUT/bench_c3_$r.$i.json 2>/dev/null
done; done
for f in $OUT/bench_*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done > $OUT/summary.txt
