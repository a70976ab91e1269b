#!/bin/bash
# r06bl: prenorm ln_dwconv tile height (VASR_OPT_DW_ROWS 8 / 16; auto picks 16 at C2 and C4) on the in-tree library.
set -uo pipefail
O=gpurun_out/r06bl; mkdir -p $O
export TMPDIR=/tmp
L=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
DW_PRENORM=1 timeout -k 10 300 python -u tools/dw_ab_libs.py 8 32:501,32:1501 $L@16 $L@8 $L@4 > $O/dw_rows.txt 2>&1 || { echo "rc $?"; tail -5 $O/dw_rows.txt; exit 1; }
grep -v amdgpu.ids $O/dw_rows.txt
