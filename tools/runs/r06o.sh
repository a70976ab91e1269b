#!/bin/bash
# r06o: what the fp32 gated tail waits on: ablations of its 36 tail steps (results wrong by design):
# 1 no weight loads after the prologue, 2 no MFMAs, 4 no A-fragment LDS reads; vs HEAD, interleaved.
set -uo pipefail
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 5 16032 f32 $V/tailg_swap1.so $V/tail_abl1.so $V/tail_abl2.so $V/tail_abl4.so > $O/ablate_f32.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ablate_f32.txt; exit 1; }
cat $O/ablate_f32.txt
timeout -k 10 300 python -u tools/tail_ab_libs.py 5 16032 bf16 $V/tailg_swap1.so $V/tail_abl1.so $V/tail_abl2.so $V/tail_abl4.so > $O/ablate_bf16.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ablate_bf16.txt; exit 1; }
cat $O/ablate_bf16.txt
