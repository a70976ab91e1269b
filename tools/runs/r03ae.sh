#!/bin/bash
# r03ae: streaming vs chunk-parallel scan at small launches over L (B = 1, 2, 4; N = 32, 64) for the
# launch-form rule of ops._use_chunked.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
for N in 32 64; do
  for B in 1 2 4; do
    for L in 32 64 128 187 256 384 501 1501; do
      for f in streaming chunked; do
        timeout -k 10 60 python tools/scan_bench.py $B $L 384 $N 2 20 $f >> $O/forms.txt 2>&1
      done
    done
  done
done
echo done > $O/DONE
