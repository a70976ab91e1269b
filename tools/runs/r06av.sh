#!/bin/bash
# r06av: the global SSM blocks' scan (N = 32, 32 clips x 64 pooled steps; gated) with 2 states per lane
# (VASR_OPT_SCAN_LANES = 2: twice the waves) and 16-step chunks vs the launcher's choice.
set -uo pipefail
O=gpurun_out/r06av; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
SCAN_N=32 timeout -k 10 300 python -u tools/scan_ab_libs.py 8 32:64,16:64 $V/head.so $V/head.so@0=2 $V/head.so@1=16 "$V/head.so@0=4" > $O/glob_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/glob_ab.txt; exit 1; }
cat $O/glob_ab.txt
