#!/bin/bash
# r06m: where the gated tail's time goes (phase stamps, f32 + bf16), then its W_z prefetch depth A/B.
set -uo pipefail
O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
VASR_LIB=$PWD/$V/tail_stamps.so timeout -k 10 120 python -u tools/diag/tail_stamps.py 16032 f32 > $O/stamps_f32.txt 2>&1 || { echo "stamps rc $?"; tail -5 $O/stamps_f32.txt; exit 1; }
cat $O/stamps_f32.txt
VASR_LIB=$PWD/$V/tail_stamps.so timeout -k 10 120 python -u tools/diag/tail_stamps.py 16032 bf16 > $O/stamps_bf16.txt 2>&1 || { echo "stamps rc $?"; tail -5 $O/stamps_bf16.txt; exit 1; }
cat $O/stamps_bf16.txt
timeout -k 10 300 python -u tools/tail_ab_libs.py 6 16032,8016 f32 $V/tailg_zpd2.so $V/tailg_zpd4.so $V/tailg_zpd6.so > $O/zpd_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/zpd_ab.txt; exit 1; }
cat $O/zpd_ab.txt
