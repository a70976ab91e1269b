#!/bin/bash
# MFMA utilisation of the projection GEMMs: one kernel-trace pass for
# durations and one PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_BF16,
# SQ_INSTS_VALU_MFMA_BF16, GRBM_GUI_ACTIVE: 3 SQ + 1 GRBM slots) over tools/gemm_pmc.py.
# Usage (repo root, via gpurun): bash tools/pmc_mfma.sh <tag> [M]
set -euo pipefail
TAG=${1:-r02}
M=${2:-8016}
OUT=gpurun_out/mfma_${TAG}_${M}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 tools/gemm_pmc.py $M > "$OUT/trace.out" 2> "$OUT/trace.err"
timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_BF16 GRBM_GUI_ACTIVE \
    -d "$OUT/pmc" -o run --output-format csv -- python3 tools/gemm_pmc.py $M > "$OUT/pmc.out" 2> "$OUT/pmc.err"
cp gpurun_out/gemm_pmc_order_${M}.json "$OUT/order.json"
echo done > "$OUT/DONE"
