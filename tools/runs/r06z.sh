#!/bin/bash
# r06z: finer phase stamps of the gated tail (out_proj steps / x1 scratch / LayerNorm / FFN1 halves), f32 + bf16.
set -uo pipefail
O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp
for k in f32 bf16; do
VASR_LIB=$PWD/tools/_variants/tail_stamps3.so timeout -k 10 120 python -u tools/diag/tail_stamps.py 16032 $k > $O/stamps_$k.txt 2>&1 || { echo "stamps rc $?"; tail -5 $O/stamps_$k.txt; exit 1; }
cat $O/stamps_$k.txt
done
