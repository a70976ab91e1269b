#!/bin/bash
# r06j: SQ counters of the fused tails (plain and gated) at M = 16032: is the tail bound by LDS (every wave
# re-reads the A operand for its one 16-column tile) or by the weight stream?
set -uo pipefail
export TMPDIR=/tmp
bash tools/pmc_kernel.sh r06j_tail python3 tools/gemm_pmc.py 16032 || { echo "pmc rc $?"; exit 1; }
for k in ssm_tail_kernel ssm_tail_gated_kernel; do echo "== $k"; python3 tools/pmc_means.py gpurun_out/pmc_r06j_tail $k; done
