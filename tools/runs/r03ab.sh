#!/bin/bash
# r03ab: packed y contraction (4 states per lane: pk_mul + pk_fma + add instead of 4 scalar FMAs; a different
# summation order), wave-major x*dt slab: bitwise A/B vs r03 HEAD lib (2-per-lane and recurrence cases must stay
# equal), GPU suite, graph-timed scan, e2e A/B.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
VASR_LIB=tools/_variants/base_r03.so timeout -k 10 300 python tools/scan_bitwise.py dump $O/base.npz > $O/bitwise.txt 2>&1
timeout -k 10 300 python tools/scan_bitwise.py dump $O/new.npz >> $O/bitwise.txt 2>&1
timeout -k 10 60 python tools/scan_bitwise.py compare $O/base.npz $O/new.npz >> $O/bitwise.txt 2>&1 || true
rm -f $O/base.npz $O/new.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for B in 16 32; do
  for v in "4 32" "4 16" "2 32" "2 16"; do
    set -- $v
    echo "npl=$1 T=$2" >> $O/scan.txt
    VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan.txt 2>&1
    VASR_LIB=tools/_variants/base_r03.so VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan_base.txt 2>&1
  done
done
timeout -k 10 900 python tools/ab_matrix.py $O/ab 2 'base|VASR_LIB=tools/_variants/base_r03.so|' 'new||' 'new_npl2t32|VASR_SCAN_NPL=2 VASR_SCAN_T=32|' > $O/ab.txt 2>&1
echo done > $O/DONE
