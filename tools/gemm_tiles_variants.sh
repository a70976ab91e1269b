#!/bin/bash
# Time the tile GEMM of every library variant in tools/_variants/ on the model's shapes
# (tools/gemm_engine_bench.py tiles column; VASR_LIB selects the library).
set -e
echo "base"; timeout -k 10 120 python tools/gemm_engine_bench.py tiles
for lib in tools/_variants/*.so; do
  echo "$(basename $lib .so)"; VASR_LIB=$PWD/$lib timeout -k 10 120 python tools/gemm_engine_bench.py tiles
done
