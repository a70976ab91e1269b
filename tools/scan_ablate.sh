#!/bin/bash
# Diagnostic: build variants of the scan kernel as separate libraries (tools/_ablate/) and time
# them with tools/scan_ablate_run.py.  VARIANTS="name:flags ..." (defaults below).
set -e
cd "$(dirname "$0")/../velocity-asr_amd"
OUT=../tools/${VARIANT_DIR:-_variants}
rm -rf $OUT && mkdir -p $OUT
VARIANTS=${VARIANTS:-"w3:-DVASR_SCAN_WAVES=3 w2:-DVASR_SCAN_WAVES=2 w4:-DVASR_SCAN_WAVES=4 noexp:-DVASR_SCAN_ABLATE=1"}
i=0
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include ${flags//,/ } \
     -fno-slp-vectorize -ffp-contract=off -shared csrc/scan.hip csrc/scan_n16.hip csrc/scan_n32.hip csrc/scan_n64.hip \
     csrc/scan_n128.hip csrc/common.cpp -o $OUT/lib_${i}_${name}.so &
  i=$((i+1))
done
wait
