#!/bin/bash
# r06x: scan wave-priority end-of-sequence variants on the ungated kernel: youth only in the last eighth
# (VASR_SCAN_PRIO=7) / from 5/8 on (8) vs HEAD (4: last quarter); rotated + warmed A/B, 32 x 10 s and 32 x 30 s.
set -uo pipefail
O=gpurun_out/r06x; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
SCAN_UNGATED=1 timeout -k 10 600 python -u tools/scan_ab_libs.py 8 32:501,32:1501 $V/scan_prio4.so $V/scan_prio7.so $V/scan_prio8.so > $O/prio_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/prio_ab.txt; exit 1; }
cat $O/prio_ab.txt
