#!/bin/bash
# r06b: z-in-tail diagnostics (which intermediate differs; isolated times), then the rest of the GPU suite.
set -uo pipefail
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag/zt_diag.py 9 501 > $O/diag_9.txt 2>&1 || { echo "diag rc $?"; tail -20 $O/diag_9.txt; exit 1; }
timeout -k 10 200 python tools/diag/zt_diag.py 32 501 > $O/diag_32.txt 2>&1 || { echo "diag rc $?"; tail -20 $O/diag_32.txt; exit 1; }
cat $O/diag_9.txt $O/diag_32.txt | grep -v amdgpu.ids
