#!/bin/bash
# r06u: gated tail with its own loads (x rows, constants, first weight steps) issued before the z product
# vs after the gate: bitwise check + interleaved A/B (f32, bf16) + phase stamps of the new form.
set -uo pipefail
O=gpurun_out/r06u; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 8 16032,8016 f32 $V/tailg_early0.so $V/tailg_early1.so > $O/early_ab_f32.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/early_ab_f32.txt; exit 1; }
cat $O/early_ab_f32.txt
timeout -k 10 300 python -u tools/tail_ab_libs.py 8 16032 bf16 $V/tailg_early0.so $V/tailg_early1.so > $O/early_ab_bf16.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/early_ab_bf16.txt; exit 1; }
cat $O/early_ab_bf16.txt
VASR_LIB=$PWD/$V/tail_stamps2.so timeout -k 10 120 python -u tools/diag/tail_stamps.py 16032 f32 > $O/stamps_f32.txt 2>&1 || { echo "stamps rc $?"; tail -5 $O/stamps_f32.txt; exit 1; }
cat $O/stamps_f32.txt
