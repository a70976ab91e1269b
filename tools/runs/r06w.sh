#!/bin/bash
# r06w: the scan's wave-priority policies re-measured on the ungated kernel (the z-in-tail default):
# 0 off, 1 time rotation, 3 fewer-chunks-first by quarter, 4 HEAD (quarters, last quarter by youth);
# rotated + warmed A/B at 32 x 10 s and 32 x 30 s.
set -uo pipefail
O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
SCAN_UNGATED=1 timeout -k 10 600 python -u tools/scan_ab_libs.py 8 32:501,32:1501 $V/scan_prio4.so $V/scan_prio0.so $V/scan_prio1.so $V/scan_prio3.so > $O/prio_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/prio_ab.txt; exit 1; }
cat $O/prio_ab.txt
