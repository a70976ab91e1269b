#!/bin/bash
# r03w: rows engine LDS footprint vs the other utterance group's scan: e2e A/B (tiles, rows d2 w8 = default,
# rows d1 w8, rows d1 w4) + isolated shapes
set -euo pipefail
O=gpurun_out/r03w
mkdir -p $O
export GEMM_SHAPES=head_comp,in_proj GEMM_ENGINES=1,2
timeout -k 10 120 python tools/gemm_engines.py > $O/eng.txt 2>&1
for v in d1 d1w4; do GEMM_ENGINES=2 VASR_LIB=tools/_variants/rows_$v.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1; done
timeout -k 10 1000 python tools/ab_matrix.py $O/ab 2 'tiles|VASR_GEMM_ENGINE=1|' 'rows_d2w8||' "rows_d1w8|VASR_LIB=tools/_variants/rows_d1.so|" "rows_d1w4|VASR_LIB=tools/_variants/rows_d1w4.so|" > $O/ab.txt 2>&1
echo done > $O/DONE
