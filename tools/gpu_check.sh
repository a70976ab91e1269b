#!/bin/bash
# GPU parity suite + smoke + default bench line on the box (repo root, via gpurun).
# Usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
set -euo pipefail
TAG=${1:-r02}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo done > gpurun_out/DONE_$TAG
