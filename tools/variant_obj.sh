#!/bin/bash
# Diagnostic: the library with ONE source rebuilt with extra flags (the other objects reused
# from velocity-asr_amd/build/), as tools/_variants/<name>.so for VASR_LIB=<path> A/B runs.
#   tools/variant_obj.sh <name> <source basename, e.g. gemm_rows.hip> [-DFLAG=...]...
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../velocity-asr_amd"
OUT=../tools/_variants/$NAME; mkdir -p "$OUT"
extra=""; case "$SRC" in scan*) extra="-fno-slp-vectorize -ffp-contract=off";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -munsafe-fp-atomics $extra "$@" \
    -c "csrc/$SRC" -o "$OUT/$SRC.o"
objs=$(ls build/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/_variants/$NAME.so $objs "$OUT/$SRC.o"
rm -rf "$OUT"
echo tools/_variants/$NAME.so
