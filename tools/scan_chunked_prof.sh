#!/bin/bash
# Per-phase times of the chunk-parallel scan (rocprofv3 kernel trace) vs the streaming kernel
# at one-utterance shapes.  Usage: bash tools/scan_chunked_prof.sh <tag>
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/scanch_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in 501 1501; do
  for npl in 2 4; do
    for ch in 0 1; do
      VASR_SCAN_NPL=$npl VASR_SCAN_CHUNKED=$ch timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/L${L}_npl${npl}_ch${ch} -o run \
        --output-format csv -- python3 tools/scan_bench.py 1 $L 384 64 2 200 > $OUT/L${L}_npl${npl}_ch${ch}.txt 2>&1
    done
  done
done
