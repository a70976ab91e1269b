#!/bin/bash
# r03i: rows GEMM engine ablations (isolated head GEMM shapes)
set -euo pipefail
O=gpurun_out/r03i
mkdir -p $O
export GEMM_SHAPES=head_comp,head_comp_b1,ctc_argmax GEMM_ENGINES=2
timeout -k 10 120 python tools/gemm_engines.py > $O/eng.txt 2>&1
for v in nomfma nostore nodma nobar nodma_nostore w8; do
  VASR_LIB=tools/_variants/rows_$v.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
done
echo done > $O/DONE
