#!/bin/bash
# r06q: what the rows-engine projection waits on at M = 16032, N = 896 (ablations, results wrong by design):
# 1 no MFMA, 2 no epilogue stores, 4 no LDS-DMA after the first two chunks, 8 no per-chunk barrier.
set -uo pipefail
O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 5 16032:896:512 $V/rows_stag0.so $V/rows_abl1.so $V/rows_abl2.so $V/rows_abl4.so $V/rows_abl8.so > $O/ablate.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ablate.txt; exit 1; }
cat $O/ablate.txt
