#!/bin/bash
# Log-mel normalisation: statistics formed inside the norm blocks for B <= 2 (one launch fewer) and
# one-round chunk staging.  GPU suite, front-end timings per library, interleaved B = 1 and C2 lines.
set -uo pipefail
OUT=gpurun_out/r05ay; mkdir -p $OUT; rm -f $OUT/frontend.txt
MAIN=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
true
true
for lib in $MAIN tools/_variants/melnofuse.so tools/_variants/melold.so; do
  for B in 1 32; do
    VASR_LIB=$lib timeout -k 10 90 python tools/frontend_bench.py $B 2>/dev/null | sed "s/^/$(basename $lib .so) B=$B /" >> $OUT/frontend.txt
  done
done
for r in 1 2 3; do
  for lib in $MAIN tools/_variants/melnofuse.so tools/_variants/melold.so; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 200 --warmup 20 \
      --no-cpu-baseline --roofline-steps 2 > $OUT/b1.$n.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/b1.$n.$r.json'));print('b1 $n r$r', d['ms_per_step'])" >> $OUT/summary.txt
  done
done
for r in 1 2; do
  for lib in $MAIN tools/_variants/melold.so; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$n.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/c2.$n.$r.json'));print('c2 $n r$r', d['value'], d['ms_per_step'])" >> $OUT/summary.txt
  done
done
cat $OUT/frontend.txt $OUT/summary.txt
