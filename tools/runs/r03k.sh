#!/bin/bash
# r03k: rows GEMM engine store groups (SUPER chunks per epilogue burst) vs tiles, bitwise-checked
set -euo pipefail
O=gpurun_out/r03k
mkdir -p $O
export GEMM_SHAPES=head_comp,head_comp_32,head_comp_b1,ctc_argmax,in_proj GEMM_ENGINES=1,2
timeout -k 10 120 python tools/gemm_engines.py > $O/eng.txt 2>&1
export GEMM_ENGINES=2
for v in s1w8 s1w8c s1w4 s2w4 s4w4; do
  VASR_LIB=tools/_variants/rows_$v.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
done
echo done > $O/DONE
