#!/bin/bash
# r06n: gated tail with z^T (operand swap: float4 y loads, 8-B gate stores, u loads first) vs before:
# bitwise check + interleaved A/B (f32, bf16), phase stamps of the new form, the tail tests.
set -uo pipefail
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 6 16032,8016 f32 $V/tailg_swap0.so $V/tailg_swap1.so > $O/swap_ab_f32.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/swap_ab_f32.txt; exit 1; }
cat $O/swap_ab_f32.txt
timeout -k 10 300 python -u tools/tail_ab_libs.py 6 16032 bf16 $V/tailg_swap0.so $V/tailg_swap1.so > $O/swap_ab_bf16.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/swap_ab_bf16.txt; exit 1; }
cat $O/swap_ab_bf16.txt
VASR_LIB=$PWD/$V/tail_stamps1.so timeout -k 10 120 python -u tools/diag/tail_stamps.py 16032 f32 > $O/stamps_f32.txt 2>&1 || { echo "stamps rc $?"; tail -5 $O/stamps_f32.txt; exit 1; }
cat $O/stamps_f32.txt
timeout -k 10 400 python -u -m pytest tests/test_ssm_tail.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tail_tests.txt 2>&1; rc=$?
tail -2 $O/tail_tests.txt; exit $rc
