#!/bin/bash
# Row-kernel variants (layer_norm rows per wave, ln_dwconv wave-tiled / tile heights): isolated
# timings + output digests at B = 1 / 16 / 32 for every library, then interleaved C2 bench lines.
set -euo pipefail
OUT=gpurun_out/r05at; mkdir -p $OUT
LIBS="velocity-asr_amd/velocity_asr/lib/libvasr_hip.so tools/_variants/wave4.so tools/_variants/wave8.so tools/_variants/wave16.so tools/_variants/lnrpw2.so tools/_variants/lnrpw4.so tools/_variants/dwtt8.so tools/_variants/dwtt32.so"
for r in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 90 python tools/rowops_bench.py 2>&1 | sed "s/^/$n r$r /" >> $OUT/rowops.txt
  done
done
cat $OUT/rowops.txt
