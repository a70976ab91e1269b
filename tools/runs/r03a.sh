#!/bin/bash
# r03a: HEAD baseline on this round's box + MFMA counters of the HEAD GEMM/tail kernels
#  + the kernels inside one graphed bench step (item 6).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
bash tools/pmc_mfma.sh r03a 8016
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/gc -o run --output-format csv -- python3 tools/graph_copies.py > $O/gc.out 2> $O/gc.err
echo done > $O/DONE
