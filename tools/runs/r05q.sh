#!/bin/bash
# r05q: the scan's workgroups per CU -- entry order and duration (stamped build), after bench-like load.
set -uo pipefail
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/scan_stamps.so timeout -k 10 200 python -u tools/diag/scan_clock.py 6 200 20 > $O/clock1.txt 2>&1 || { echo "clock1 rc $?"; tail -5 $O/clock1.txt; exit 1; }
cat $O/clock1.txt
