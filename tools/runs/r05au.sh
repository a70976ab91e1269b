#!/bin/bash
# ln_dwconv tile height by launch size (VASR_OPT_DW_ROWS): parity + bitwise tests, isolated
# timings per forced height, then interleaved one-utterance (10 s) and C2 lines, auto vs 16 rows.
set -euo pipefail
OUT=gpurun_out/r05au; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_host.py -x -q --timeout 120 --timeout-method thread -k "dwconv or layer_norm or option" > $OUT/pytest.txt 2>&1
for rows in 16 8 4 0; do
  VASR_DW_ROWS=$rows timeout -k 10 90 python tools/rowops_bench.py 2>/dev/null | sed "s/^/rows=$rows /" >> $OUT/rowops.txt
done
for r in 1 2 3; do
  for rows in 16 0; do
    VASR_DW_ROWS=$rows timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 200 --warmup 20 \
      --no-cpu-baseline --roofline-steps 2 > $OUT/b1.$rows.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/b1.$rows.$r.json'));print('b1 rows=$rows r$r', d['ms_per_step'])" >> $OUT/summary.txt
  done
done
for r in 1 2; do
  for rows in 16 0; do
    VASR_DW_ROWS=$rows timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$rows.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/c2.$rows.$r.json'));print('c2 rows=$rows r$r', d['value'], d['ms_per_step'])" >> $OUT/summary.txt
  done
done
cat $OUT/rowops.txt $OUT/summary.txt; tail -3 $OUT/pytest.txt
