#!/bin/bash
# Diagnostic: build the whole library with extra compile flags into tools/_variants/<name>.so,
# for A/B timing through VASR_LIB=<path> (velocity_asr/_lib.py).
#   tools/build_variant_lib.sh <name> [-DFLAG=...]...
# EXTRA_<source stem>="flags" adds flags to one source file only (EXTRA_stft="-fno-slp-vectorize").
set -e
NAME=$1; shift
cd "$(dirname "$0")/../velocity-asr_amd"
OUT=../tools/_variants/$NAME; mkdir -p "$OUT"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -munsafe-fp-atomics $*"
for f in csrc/*.hip csrc/*.cpp; do
  extra=""; case "$(basename $f)" in scan*.hip) extra="-fno-slp-vectorize -ffp-contract=off";; stft.hip) extra="-fno-slp-vectorize";; esac
  stem=$(basename $f); stem=${stem%.*}; v="EXTRA_$stem"; extra="$extra ${!v:-}"
  /opt/rocm/bin/hipcc $FLAGS $extra -c "$f" -o "$OUT/$(basename $f).o" &
  pids="$pids $!"
done
for p in $pids; do wait $p; done  # set -e: a failed compile ends the script
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/_variants/$NAME.so "$OUT"/*.o
rm -rf "$OUT"
echo ../tools/_variants/$NAME.so
