#!/bin/bash
# Global context: norm2 -> q projection and the fusion's local product on a side stream beside the
# pooled global chain (VASR_CTX_OVERLAP=1, default) vs one stream (=0).  GPU suite, then interleaved lines.
set -uo pipefail
OUT=gpurun_out/r05ba; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for ov in 0 1; do
    VASR_CTX_OVERLAP=$ov timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$ov.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/c2.$ov.$r.json'));s=d['config']['schedule'];print('c2 ov=$ov r$r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['tokens_vs_reference']['all_ranks_pass'])" >> $OUT/summary.txt
  done
done
for r in 1 2 3; do
  for ov in 0 1; do
    VASR_CTX_OVERLAP=$ov timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 200 --warmup 20 \
      --no-cpu-baseline --roofline-steps 2 > $OUT/b1.$ov.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b1.$ov.$r.json'));print('b1 ov=$ov r$r', d['ms_per_step'])" >> $OUT/summary.txt
  done
done
for ov in 0 1; do
  VASR_CTX_OVERLAP=$ov timeout -k 10 300 python bench.py --no-cpu-baseline --no-scatter --seconds 30 > $OUT/c4.$ov.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/c4.$ov.json'));s=d['config']['schedule'];print('c4 ov=$ov', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['tokens_vs_reference']['all_ranks_pass'])" >> $OUT/summary.txt
done
cat $OUT/summary.txt
