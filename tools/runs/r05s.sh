#!/bin/bash
# r05s: per-CU balance of the scan's three blocks under wave-priority rotation (stamped builds), and timing of
# the rotation variants (time phases 2^14/15/16 cycles, chunk-index phases, descending by progress).
set -uo pipefail
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
for v in scan_stamps stamps_p15 stamps_pchunk stamps_pdesc; do
VASR_LIB=tools/_variants/$v.so timeout -k 10 200 python -u tools/diag/scan_clock.py 4 200 20 > $O/clock_$v.txt 2>&1 || { echo "$v rc $?"; tail -5 $O/clock_$v.txt; exit 1; }
echo "== $v"; tail -8 $O/clock_$v.txt
done
for b in 32 16; do
SCAN_MODES=2 SCAN_B=$b VARIANT_DIR=_abl8 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$b.txt 2>&1 || { echo "b$b rc $?"; tail -5 $O/b$b.txt; exit 1; }
cat $O/b$b.txt
done
