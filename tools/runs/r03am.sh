#!/bin/bash
# r03am: is the world-1 RCCL graphed-transcription mismatch of r03al flaky or tied to VASR_ROWS_VST?
set -uo pipefail
O=gpurun_out/r03am
mkdir -p $O
T=tests/test_distributed_gpu.py::test_rccl_sharded_transcription_world1_matches_reference
for v in 1 0 1 0; do
  VASR_ROWS_VST=$v timeout -k 10 200 python -u -m pytest $T -x -q --timeout 150 --timeout-method thread > $O/t_$v.txt 2>&1
  echo "VST=$v rc=$? $(tail -1 $O/t_$v.txt)" >> $O/res.txt
done
cat $O/res.txt
