#!/bin/bash
# r03t: rows engine with whole-chunk softplus branches (isolated, bitwise vs tiles)
set -euo pipefail
O=gpurun_out/r03t
mkdir -p $O
export GEMM_SHAPES=head_comp,head_comp_32,in_proj,ffn1_192 GEMM_ENGINES=1,2
timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
GEMM_ENGINES=2 VASR_LIB=tools/_variants/rows_nost.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
echo done > $O/DONE
