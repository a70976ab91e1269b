#!/bin/bash
# r03ad: HBM write bandwidth of the projection GEMM's C pattern vs other layouts (tools/ubench/store_pattern),
# scan launch time over the batch size (waves per SIMD: 4 states per lane, automatic chunk length).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 60 ./tools/ubench/store_pattern > $O/store_pattern.txt 2>&1
for B in 4 8 10 11 12 14 16 18 21 22 24 32; do
  timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 30 >> $O/scan_bsweep.txt 2>&1
done
echo done > $O/DONE
