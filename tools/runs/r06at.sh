#!/bin/bash
# r06at: the global SSM blocks' projection (M = 2048, N = 1280) and the C2 / C4 shapes on the rows engine
# forced (VASR_OPT_GEMM_ENGINE = 2) vs the picker.
set -uo pipefail
O=gpurun_out/r06at; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 6 2048:1280:896,4096:1280:896,1024:1280:896 $V/head.so $V/head.so@3=2 $V/head.so@3=1 > $O/engine_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/engine_ab.txt; exit 1; }
cat $O/engine_ab.txt
