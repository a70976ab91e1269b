#!/bin/bash
# r06ay: front-end XCD-run order per kernel (VASR_FE_XCD mask: 1 STFT, 2 log-mel, 4 norm), stft+mel pair A/B.
set -uo pipefail
O=gpurun_out/r06ay; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 400 python -u tools/fe_ab_libs.py 8 32:160000,32:480000,16:160000 $V/fexcd0.so $V/fexm1.so $V/fexm2.so $V/fexm4.so $V/fexm6.so $V/fexcd1.so > $O/fe_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/fe_ab.txt; exit 1; }
cat $O/fe_ab.txt
