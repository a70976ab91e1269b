#!/bin/bash
# r03aa: where the scan's time goes after the cheaper butterfly + x*dt pre-pass: ablations (diagnostic builds,
# tools/_ablate) at the 16-clip launch for both lane layouts (32-step chunks), and SQ counters of the new kernels.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
for v in "2 32" "4 32" "4 16"; do
  set -- $v
  echo "npl=$1 T=$2 B=16" >> $O/ablate.txt
  VARIANT_DIR=_ablate SCAN_B=16 SCAN_MODES=2 VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 120 python tools/scan_ablate_run.py >> $O/ablate.txt 2>&1
done
VASR_SCAN_NPL=2 VASR_SCAN_T=32 bash tools/pmc_kernel.sh r03aa_npl2t32 python3 tools/scan_bench.py 16 501 384 64 2 20
VASR_SCAN_NPL=4 VASR_SCAN_T=32 bash tools/pmc_kernel.sh r03aa_npl4t32 python3 tools/scan_bench.py 16 501 384 64 2 20
echo done > $O/DONE
