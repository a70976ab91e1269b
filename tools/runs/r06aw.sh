#!/bin/bash
# r06aw: the 32-row tail's weight prefetch distance (VASR_TAIL_PD21: 1 / 2 HEAD / 3 with spills), gated tail.
set -uo pipefail
O=gpurun_out/r06aw; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 6 16032,8016 f32 $V/pd2.so $V/pd1.so $V/pd3.so > $O/pd_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/pd_ab.txt; exit 1; }
cat $O/pd_ab.txt
