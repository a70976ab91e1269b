#!/bin/bash
# r04ai: 32-clip scan launch -- 16-step form (default) vs the 32-step form register-limited to
# three waves per SIMD (VASR_SCAN_WAVES_TC32=3 build, 102 spilled VGPRs), forced with VASR_SCAN_T=32.
set -uo pipefail
O=gpurun_out/r04ai
mkdir -p $O
for i in 1 2; do
  timeout -k 10 100 python -u tools/scan_bench.py 32 501 384 64 2 50 > $O/t16_$i.txt 2>&1 || exit 1
  VASR_LIB=tools/_variants/t32w3.so VASR_SCAN_T=32 timeout -k 10 100 python -u tools/scan_bench.py 32 501 384 64 2 50 > $O/t32w3_$i.txt 2>&1 || exit 1
  VASR_SCAN_T=32 timeout -k 10 100 python -u tools/scan_bench.py 32 501 384 64 2 50 > $O/t32w2_$i.txt 2>&1 || exit 1
done
for f in $O/*.txt; do echo "$f: $(grep -v libdrm $f | tail -1)"; done
