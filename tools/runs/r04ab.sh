#!/bin/bash
# r04ab: rows-engine loader waves counting every younger vector-memory op (issue-order vmcnt) vs
# vmcnt(0): GEMM time (interleaved x2), cycle stamps of both, bitwise vs tiles.
set -uo pipefail
O=gpurun_out/r04ab
mkdir -p $O
for i in 1 2; do
  timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/base$i.txt 2>&1 || exit 1
  VASR_LIB=tools/_variants/lwall.so timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/lwall$i.txt 2>&1 || exit 1
done
VASR_LIB=tools/_variants/rowstamps.so timeout -k 10 100 python -u tools/diag/rows_stamps.py 8016 > $O/stamps_base.txt 2>&1 || exit 1
VASR_LIB=tools/_variants/lwallstamps.so timeout -k 10 100 python -u tools/diag/rows_stamps.py 8016 > $O/stamps_lwall.txt 2>&1 || exit 1
grep -h "M=" $O/*.txt
