#!/bin/bash
# Counters of the fused SSMBlock tail in isolation.  Usage: bash tools/tail_pmc.sh <tag>
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/tailpmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/tail_bench.py > $OUT/bench.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/tail_bench.py 8016 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d $OUT/pmc1 -o run --output-format csv -- python3 tools/tail_bench.py 8016 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d $OUT/pmc2 -o run --output-format csv -- python3 tools/tail_bench.py 8016 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum \
  -d $OUT/pmc3 -o run --output-format csv -- python3 tools/tail_bench.py 8016 > /dev/null 2>&1
