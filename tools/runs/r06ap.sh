#!/bin/bash
# r06ap: rows-engine projection with 3 W chunks in flight (VASR_ROWS_DEPTH=3, 154 KiB LDS) vs 2.
set -uo pipefail
O=gpurun_out/r06ap; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 6 16032:896:512,48032:896:512,8016:896:512 $V/rows_d2.so $V/rows_d3.so > $O/depth_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/depth_ab.txt; exit 1; }
cat $O/depth_ab.txt
