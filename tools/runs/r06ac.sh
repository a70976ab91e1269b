#!/bin/bash
# r06ac: MFMA counters at HEAD (projection GEMMs, gated tail with the transposed z product) at M = 16032.
set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_mfma.sh r06ac 16032 > gpurun_out/pmc_mfma_r06ac.log 2>&1 || { echo "rc $?"; tail -5 gpurun_out/pmc_mfma_r06ac.log; exit 1; }
echo ok
