#!/bin/bash
# r03y: SQ counters of the scan's two lane layouts at the bench's 16-clip launch (4 states per lane, 32-step
# chunks = default; 2 per lane, 32-step chunks), and the HEAD bench profile (kernel stats + HBM traffic).
set -euo pipefail
export TMPDIR=/tmp
VASR_SCAN_NPL=4 VASR_SCAN_T=32 bash tools/pmc_kernel.sh r03y_npl4t32 python3 tools/scan_bench.py 16 501 384 64 2 20
VASR_SCAN_NPL=2 VASR_SCAN_T=32 bash tools/pmc_kernel.sh r03y_npl2t32 python3 tools/scan_bench.py 16 501 384 64 2 20
bash tools/profile.sh r03y
echo done > gpurun_out/r03y_DONE
