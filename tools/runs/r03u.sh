#!/bin/bash
# r03u: rows engine with the epilogue interleaved into the next chunk's MFMAs (4 waves default; 8-wave variant)
set -euo pipefail
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rows_engine" > $O/pytest.txt 2>&1
export GEMM_SHAPES=head_comp,head_comp_32,ctc_argmax,in_proj,ffn1_192 GEMM_ENGINES=1,2
timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
GEMM_ENGINES=2 VASR_LIB=tools/_variants/rows_i8.so timeout -k 10 120 python tools/gemm_engines.py >> $O/eng.txt 2>&1
echo done > $O/DONE
