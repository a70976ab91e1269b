#!/bin/bash
# r03ac: y partial sums through a per-wave LDS tile (4 states per lane, N = 64, full chunks), summed in the
# butterfly's pairing order: bitwise A/B against the same source without it (-DVASR_SCAN_LDSY=0), graph-timed
# scan, GPU suite, e2e A/B.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
VASR_LIB=tools/_variants/noldsy.so timeout -k 10 300 python tools/scan_bitwise.py dump $O/base.npz > $O/bitwise.txt 2>&1
timeout -k 10 300 python tools/scan_bitwise.py dump $O/new.npz >> $O/bitwise.txt 2>&1
timeout -k 10 60 python tools/scan_bitwise.py compare $O/base.npz $O/new.npz >> $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
for B in 16 32; do
  for v in "4 32" "4 16"; do
    set -- $v
    echo "npl=$1 T=$2" >> $O/scan.txt
    VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan.txt 2>&1
    VASR_LIB=tools/_variants/noldsy.so VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan_base.txt 2>&1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 900 python tools/ab_matrix.py $O/ab 3 'noldsy|VASR_LIB=tools/_variants/noldsy.so|' 'ldsy||' > $O/ab.txt 2>&1
echo done > $O/DONE
