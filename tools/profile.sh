#!/bin/bash
# rocprofv3 passes over bench.py on the GPU box (run from the repo root via gpurun):
#   1. kernel trace + stats (per-kernel average durations)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate PMC passes; TCC slot limits)
# Output: gpurun_out/prof_<tag>/...   Usage: tools/profile.sh <tag> [bench args]
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${*:---steps 10 --warmup 3 --no-cpu-baseline}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --inproc $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --inproc --steps 2 --warmup 1 --no-cpu-baseline --roofline-steps 1 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --inproc --steps 2 --warmup 1 --no-cpu-baseline --roofline-steps 1 > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo done > "$OUT/DONE"
