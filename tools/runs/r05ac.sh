#!/bin/bash
# r05ac: upper-stack levels held in registers: 5 (HEAD), 3, 0 (the rest in LDS); scan launch times.
set -uo pipefail
O=gpurun_out/r05ac
mkdir -p $O
export TMPDIR=/tmp
for bl in "32 501" "16 501" "32 1501"; do
set -- $bl
SCAN_MODES=2 SCAN_B=$1 SCAN_L=$2 VARIANT_DIR=_abl10 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$1_l$2.txt 2>&1 || { echo "b$1 rc $?"; tail -5 $O/b$1_l$2.txt; exit 1; }
echo "B=$1 L=$2"; cat $O/b$1_l$2.txt
done
