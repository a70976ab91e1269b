#!/bin/bash
# r03q: rows engine store/DMA ordering variants (isolated, bitwise-checked vs tiles)
set -euo pipefail
O=gpurun_out/r03q
mkdir -p $O
export GEMM_SHAPES=head_comp,head_comp_32,in_proj GEMM_ENGINES=2
for v in base if nsw ifnsw nostore base; do
  VASR_LIB=tools/_variants/rows_$v.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
done
echo done > $O/DONE
