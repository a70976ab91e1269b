#!/bin/bash
# Full GPU check of the tree on the box: parity suite, smoke, bench line, rocprofv3 passes.
# Usage (via gpurun, repo root): bash tools/round_check.sh <tag>
set -euo pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
bash tools/profile.sh $TAG
