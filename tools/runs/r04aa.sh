#!/bin/bash
# r04aa: rows-engine ablations at the bench shapes (1 no MFMA, 2 no stores, 4 no DMA after the
# first chunks, 5 = stores only, 6 = MFMA only), times only (results are garbage by design).
set -uo pipefail
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/base.txt 2>&1 || exit 1
for a in 1 2 4 5 6; do
  VASR_LIB=tools/_variants/rowsab$a.so timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/ab$a.txt 2>&1 || { echo "ab$a rc $?"; exit 1; }
done
grep -h "M=" $O/*.txt
