#!/bin/bash
# r05n: scan compiled under other machine-scheduler strategies (tools/scan_variants_build.sh), B=32 and B=16, mode 2.
set -uo pipefail
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
for b in 32 16; do
SCAN_MODES=2 SCAN_B=$b VARIANT_DIR=_abl6 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$b.txt 2>&1 || { echo "b$b rc $?"; tail -5 $O/b$b.txt; exit 1; }
cat $O/b$b.txt
done
