#!/bin/bash
# r06g: one 12-wave scan workgroup per CU vs three 4-wave ones (VASR_OPT_SCAN_WG = 7): bitwise (every scan
# case), interleaved launch times at C2 / C4 shapes; the C4 cache A/B again with rotated order.
set -uo pipefail
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/scan_bitwise.py dump $O/wg4.npz > $O/dump4.txt 2>&1 || { echo "dump rc $?"; tail -5 $O/dump4.txt; exit 1; }
VASR_SCAN_WG=12 timeout -k 10 300 python tools/scan_bitwise.py dump $O/wg12.npz > $O/dump12.txt 2>&1 || { echo "dump12 rc $?"; tail -5 $O/dump12.txt; exit 1; }
python tools/scan_bitwise.py compare $O/wg4.npz $O/wg12.npz > $O/bitwise.txt 2>&1; tail -2 $O/bitwise.txt
rm -f $O/wg4.npz $O/wg12.npz
L=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
timeout -k 10 500 python tools/scan_ab_libs.py 6 32:501,32:1501 $L@7=4 $L@7=12 tools/_variants_scan/lib_2_nocache.so tools/_variants/base_r06.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
