#!/bin/bash
# SQ counters of the 32- and 16-clip scan launches at the final HEAD (two --pmc passes each).
set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_kernel.sh r05az_scan32 python3 tools/scan_bench.py 32 501 384 64 2 50 || { echo "pmc32 rc $?"; exit 1; }
timeout -k 10 400 bash tools/pmc_kernel.sh r05az_scan16 python3 tools/scan_bench.py 16 501 384 64 2 50 || { echo "pmc16 rc $?"; exit 1; }
python3 tools/pmc_means.py gpurun_out/pmc_r05az_scan32 ssm_scan_kernel 501 > gpurun_out/pmc_r05az_scan32/means.txt
python3 tools/pmc_means.py gpurun_out/pmc_r05az_scan16 ssm_scan_kernel 501 > gpurun_out/pmc_r05az_scan16/means.txt
cat gpurun_out/pmc_r05az_scan32/means.txt gpurun_out/pmc_r05az_scan16/means.txt
