#!/bin/bash
# One bench line per BASELINE config on one box (same HEAD): C2 fp32 32x10 s (default), C3 bf16
# per-GPU shape, C4 32x30 s, C5 INT8, plus one-utterance latency (B=1, 10 s and 30 s).
# Usage: bash tools/config_benches.sh <tag>
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/cfg_$TAG
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err; }
run c2
run c3_bf16 --bf16
run c4_30s --seconds 30
run c5_int8 --int8
run b1_10s --batch 1 --steps 50 --warmup 10
run b1_30s --batch 1 --seconds 30 --steps 50 --warmup 10
