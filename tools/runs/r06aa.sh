#!/bin/bash
# r06aa: the tail's LayerNorm with each wave's rows interleaved (loads first, reductions side by side) vs
# one row after another: bitwise check + interleaved A/B of the gated tail (f32, bf16); finer stamps;
# the tail tests (row forms bitwise, fused vs unfused, z-in-tail).
set -uo pipefail
O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 8 16032,8016,4097 f32 $V/ln_old.so $V/ln_new.so > $O/ln_ab_f32.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ln_ab_f32.txt; exit 1; }
cat $O/ln_ab_f32.txt
timeout -k 10 300 python -u tools/tail_ab_libs.py 8 16032 bf16 $V/ln_old.so $V/ln_new.so > $O/ln_ab_bf16.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ln_ab_bf16.txt; exit 1; }
cat $O/ln_ab_bf16.txt
timeout -k 10 400 python -u -m pytest tests/test_ssm_tail.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tail_tests.txt 2>&1; rc=$?
tail -2 $O/tail_tests.txt; exit $rc
