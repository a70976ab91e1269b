#!/bin/bash
# Adaptive pool: window rows loaded 8 at a time before the in-order adds.  Bitwise test on both
# libraries, GPU suite, interleaved one-utterance and C2 lines vs the previous library.
set -uo pipefail
OUT=gpurun_out/r05bf; mkdir -p $OUT
MAIN=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
OLD=tools/_variants/poolold.so
VASR_LIB=$OLD timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "adaptive_pool" > $OUT/old_pool_tests.txt 2>&1; echo "old lib pool tests rc $?"; tail -1 $OUT/old_pool_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in $MAIN $OLD; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 200 --warmup 20 \
      --no-cpu-baseline --roofline-steps 2 > $OUT/b1.$n.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b1.$n.$r.json'));print('b1 $n r$r', d['ms_per_step'])" >> $OUT/summary.txt
  done
done
for r in 1 2; do
  for lib in $MAIN $OLD; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$n.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/c2.$n.$r.json'));print('c2 $n r$r', d['value'], d['ms_per_step'], d['tokens_vs_reference']['all_ranks_pass'])" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
