#!/bin/bash
# r05m: scan ablations at the 32-clip launch (B=32, 3 waves/SIMD, 16-step chunks) and the 16-clip one,
# mode 2; then the 32-step form forced at B=32; the counter list of the box.
set -uo pipefail
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "list rc $?"
SCAN_MODES=2 SCAN_B=32 VARIANT_DIR=_abl5 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b32.txt 2>&1 || { echo "b32 rc $?"; tail -5 $O/b32.txt; exit 1; }
cat $O/b32.txt
SCAN_MODES=2 SCAN_B=16 VARIANT_DIR=_abl5 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b16.txt 2>&1 || { echo "b16 rc $?"; exit 1; }
cat $O/b16.txt
VASR_SCAN_T=32 SCAN_MODES=2 SCAN_B=32 VARIANT_DIR=_abl5 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b32_t32.txt 2>&1 || { echo "t32 rc $?"; exit 1; }
cat $O/b32_t32.txt
