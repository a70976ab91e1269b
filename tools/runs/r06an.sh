#!/bin/bash
# r06an: tile-engine shapes forced per GEMM at the one-graph C2 shapes (temporal binding K = 240, the fusion's
# out and local products, the argmax head) vs the picker.
set -uo pipefail
O=gpurun_out/r06an; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 600 python -u tools/gemm_ab_libs.py 5 16032:192:0:240,16032:192:0:192,16032:384:0:192,16032:1000:-1:192 $V/x3_auto.so $V/x3_cfg0.so $V/x3_cfg1.so $V/x3_cfg2.so > $O/cfg_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/cfg_ab.txt; exit 1; }
cat $O/cfg_ab.txt
