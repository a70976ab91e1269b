#!/bin/bash
# r06as: tile shapes for the global SSM blocks' projection (M = 2048, N = 1280, K = 192) and the other
# small-M GEMMs (N = 384 / 192 at M = 2048, N = 96 at 512): picker vs forced 128 x 128 / 128 x 64.
set -uo pipefail
O=gpurun_out/r06as; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 6 2048:1280:896,2048:384:0,2048:192:0,512:96:0 $V/x3_auto.so $V/x3_cfg0.so $V/x3_cfg1.so > $O/cfg_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/cfg_ab.txt; exit 1; }
cat $O/cfg_ab.txt
