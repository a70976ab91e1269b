#!/bin/bash
# r06h: wave priority ranked by the sibling workgroups' chunk progress (VASR_SCAN_PRIO=6) vs the quarter
# policy (4, HEAD): bitwise (the variant library's scan cases vs HEAD's), interleaved launch times.
set -uo pipefail
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants_scan2/lib_0_prio6.so timeout -k 10 300 python tools/scan_bitwise.py dump $O/p6.npz > $O/dump6.txt 2>&1 || { echo "dump rc $?"; tail -5 $O/dump6.txt; exit 1; }
timeout -k 10 300 python tools/scan_bitwise.py dump $O/head.npz > $O/dumph.txt 2>&1 || { echo "dumph rc $?"; tail -5 $O/dumph.txt; exit 1; }
python tools/scan_bitwise.py compare $O/head.npz $O/p6.npz > $O/bitwise.txt 2>&1; tail -2 $O/bitwise.txt
rm -f $O/*.npz
timeout -k 10 500 python tools/scan_ab_libs.py 6 32:501,32:1501,16:501 tools/_variants_scan2/lib_1_prio4.so tools/_variants_scan2/lib_0_prio6.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
