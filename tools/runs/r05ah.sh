#!/bin/bash
# r05ah: refinements of the scan's "fewer chunks first" priority: last quarter by age reversed (P5), the
# youngest block one level up (P6); per-CU exits (stamped builds) and launch times.
set -uo pipefail
O=gpurun_out/r05ah
mkdir -p $O
export TMPDIR=/tmp
for v in scan_stamps stamps_p5 stamps_p6; do
VASR_LIB=tools/_variants/$v.so timeout -k 10 200 python -u tools/diag/scan_clock.py 4 200 20 > $O/clock_$v.txt 2>&1 || { echo "$v rc $?"; tail -5 $O/clock_$v.txt; exit 1; }
echo "== $v"; tail -5 $O/clock_$v.txt
done
for bl in "32 501" "32 1501"; do
set -- $bl
SCAN_MODES=2 SCAN_B=$1 SCAN_L=$2 VARIANT_DIR=_abl11 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$1_l$2.txt 2>&1 || { echo "b$1 rc $?"; tail -5 $O/b$1_l$2.txt; exit 1; }
echo "B=$1 L=$2"; cat $O/b$1_l$2.txt
done
