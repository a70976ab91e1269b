#!/bin/bash
# r03v: rows engine (8 waves, whole-chunk softplus branches): parity, isolated shapes, C2 A/B vs tiles
set -euo pipefail
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rows_engine or pinned or statedim" > $O/pytest.txt 2>&1
GEMM_SHAPES=head_comp,head_comp_32,in_proj GEMM_ENGINES=1,2 timeout -k 10 120 python tools/gemm_engines.py > $O/eng.txt 2>&1
timeout -k 10 900 python tools/ab_matrix.py $O/ab 2 'tiles|VASR_GEMM_ENGINE=1|' 'auto||' > $O/ab.txt 2>&1
echo done > $O/DONE
