#!/bin/bash
# r05d: stft.hip SLP build with 32-bit index arithmetic (C: no SDWA / packed-u16 index math, 153
# packed-fp32 ops) in the interference sequence of r05c; and the XCD of each workgroup by launch size.
set -uo pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/stft_slp_opidx.so timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 > $O/seq_C.txt 2>&1 || { echo "seq C rc $?"; tail -5 $O/seq_C.txt; exit 1; }
grep aggressor $O/seq_C.txt
timeout -k 10 120 python -u tools/diag/xcd_map.py > $O/xcd_map.txt 2>&1 || { echo "xcd rc $?"; tail -5 $O/xcd_map.txt; exit 1; }
cat $O/xcd_map.txt
