#!/bin/bash
# r06y: ln_dwconv with its workgroups per CU capped (dynamic LDS pads: two or more rounds, so one round's
# stores overlap the next round's loads) and 8-row tiles, vs HEAD, at 32 x 501 and 32 x 1501.
set -uo pipefail
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/dw_ab_libs.py 8 32:501,32:1501 $V/dw_base.so $V/dw_pad30000.so $V/dw_pad48000.so $V/dw_base.so@8 $V/dw_pad20000.so@8 $V/dw_pad30000.so@8 $V/dw_pad48000.so@8 > $O/dw_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/dw_ab.txt; exit 1; }
cat $O/dw_ab.txt
