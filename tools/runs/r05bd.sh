#!/bin/bash
# 128 x 64 tile threshold 1.4 -> 2.35 per CU (N = 192 GEMMs of the 32-clip graph on 64 x 64 tiles):
# GPU suite, then interleaved lines per config, HEAD vs the previous library (tools/_variants/x3old.so).
set -uo pipefail
OUT=gpurun_out/r05bd; mkdir -p $OUT
MAIN=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
OLD=tools/_variants/x3old.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
line() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  VASR_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-scatter "$@" > $OUT/$tag.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/$tag.json'));s=d['config'].get('schedule') or {};print('$tag', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), d['tokens_vs_reference']['all_ranks_pass'])" >> $OUT/summary.txt
}
for r in 1 2 3; do line c2.new.$r $MAIN; line c2.old.$r $OLD; done
for r in 1 2; do line c3.new.$r $MAIN --bf16; line c3.old.$r $OLD --bf16; done
line c4.new $MAIN --seconds 30; line c4.old $OLD --seconds 30
line c5.new $MAIN --int8; line c5.old $OLD --int8
cat $OUT/summary.txt
