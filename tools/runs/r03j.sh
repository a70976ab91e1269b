#!/bin/bash
# r03j: rows GEMM engine: DMA depth x waves per block x nt stores (isolated)
set -euo pipefail
O=gpurun_out/r03j
mkdir -p $O
export GEMM_SHAPES=head_comp,head_comp_32,head_comp_b1,ctc_argmax,in_proj GEMM_ENGINES=1,2
timeout -k 10 120 python tools/gemm_engines.py > $O/eng.txt 2>&1
export GEMM_ENGINES=2
for v in d3 d2w8 d3w8 d2nt d3w8nt; do
  VASR_LIB=tools/_variants/rows_$v.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
done
echo done > $O/DONE
