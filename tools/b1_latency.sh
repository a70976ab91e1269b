#!/bin/bash
# B = 1 latency (one utterance, audio -> tokens, HIP graph) with the chunk-parallel scan and
# with the streaming kernel, 10 s and 30 s clips.  Usage: bash tools/b1_latency.sh <tag>
set -euo pipefail
TAG=${1:-r02}
mkdir -p gpurun_out/b1_$TAG
for sec in 10 30; do
  for ch in 1 0; do
    VASR_SCAN_CHUNKED=$ch timeout -k 10 200 python bench.py --inproc --batch 1 --seconds $sec --steps 50 --warmup 10 \
      --no-cpu-baseline --roofline-steps 2 > gpurun_out/b1_$TAG/b1_${sec}s_chunked$ch.json 2> gpurun_out/b1_$TAG/err_${sec}_$ch.log
  done
done
