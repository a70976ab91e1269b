#!/bin/bash
# r06bf: the prenorm ln_dwconv's LayerNorm slots without per-row branches (pre_new) vs HEAD (pre_old), then the fold tests.
set -uo pipefail
O=gpurun_out/r06bf; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
DW_PRENORM=1 timeout -k 10 300 python -u tools/dw_ab_libs.py 8 32:501,32:1501,2:501 $V/pre_old.so $V/pre_new.so > $O/dw_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/dw_ab.txt; exit 1; }
cat $O/dw_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_ln_pair.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; exit $rc
