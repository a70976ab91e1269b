#!/bin/bash
# Diagnostic: build scan-only libraries (scan*.hip + common.cpp) for tools/scan_ablate_run.py, one
# translation unit per job (make -j style).  VARIANTS="name:flag,flag ..."; VARIANT_DIR (default _abl).
set -e
cd "$(dirname "$0")/../velocity-asr_amd"
OUT=../tools/${VARIANT_DIR:-_abl}
rm -rf $OUT && mkdir -p $OUT/obj
i=0
jobs=()
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  mkdir -p $OUT/obj/$i
  for f in csrc/scan.hip csrc/scan_n16.hip csrc/scan_n32.hip csrc/scan_n64.hip csrc/scan_n128.hip csrc/common.cpp; do
    echo "/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include $flags -fno-slp-vectorize -ffp-contract=off -c $f -o $OUT/obj/$i/$(basename $f).o"
  done
  i=$((i+1))
done > $OUT/cmds.txt
xargs -P ${JOBS:-8} -I{} bash -c "{}" < $OUT/cmds.txt
i=0
for v in $VARIANTS; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_${i}_${name}.so $OUT/obj/$i/*.o
  i=$((i+1))
done
rm -rf $OUT/obj
ls $OUT
