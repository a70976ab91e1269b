#!/bin/bash
# r03f: scan ablations at the bench's 16-clip launch and at 32 clips (isolated launches).
set -euo pipefail
O=gpurun_out/r03f
mkdir -p $O
SCAN_B=16 SCAN_MODES=2 VARIANT_DIR=_abl timeout -k 10 300 python tools/scan_ablate_run.py > $O/abl_b16.txt 2>&1
SCAN_B=32 SCAN_MODES=2 VARIANT_DIR=_abl timeout -k 10 300 python tools/scan_ablate_run.py > $O/abl_b32.txt 2>&1
echo done > $O/DONE
