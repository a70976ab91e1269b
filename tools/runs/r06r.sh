#!/bin/bash
# r06r: rows-engine phase stamps at the z-in-tail projection (N = 896) and the 1280-column form.
set -uo pipefail
O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp
ROWS_N=896 VASR_LIB=$PWD/tools/_variants/rowstamps.so timeout -k 10 120 python -u tools/diag/rows_stamps.py 16032 8016 > $O/stamps_896.txt 2>&1 || { echo "rc $?"; tail -5 $O/stamps_896.txt; exit 1; }
cat $O/stamps_896.txt
ROWS_N=1280 VASR_LIB=$PWD/tools/_variants/rowstamps.so timeout -k 10 120 python -u tools/diag/rows_stamps.py 16032 > $O/stamps_1280.txt 2>&1 || { echo "rc $?"; tail -5 $O/stamps_1280.txt; exit 1; }
cat $O/stamps_1280.txt
