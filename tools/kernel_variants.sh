#!/bin/bash
# Diagnostic: build variants of one kernel source as separate libraries in tools/_variants/.
#   tools/kernel_variants.sh <src.hip> "name:flag1,flag2 name2:flags ..."
set -e
SRC=$1; VARIANTS=$2
cd "$(dirname "$0")/../velocity-asr_amd"
OUT=${OUT:-_variants}
rm -rf ../tools/$OUT && mkdir -p ../tools/$OUT
i=0
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include ${flags//,/ } \
     -shared csrc/$SRC csrc/common.cpp -o ../tools/$OUT/lib_${i}_${name}.so &
  i=$((i+1))
done
wait
ls ../tools/$OUT
