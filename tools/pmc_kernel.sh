#!/bin/bash
# SQ/GRBM counter passes (separate rocprofv3 --pmc runs, kernel trace only) over a command.
#   tools/pmc_kernel.sh <tag> <command...>     -> gpurun_out/pmc_<tag>/p{1,2,3}/
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES"
i=1
for P in "$P1" "$P2"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d "$OUT/p$i" -o run --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1
  i=$((i+1))
done
echo done > "$OUT/DONE"
