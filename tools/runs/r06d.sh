#!/bin/bash
# r06d: scan changes vs the round-start library -- every scan case bitwise (tools/scan_bitwise.py), launch
# times at the C2 / C4 shapes interleaved, the C4 clock-vs-cycles question with the stamped build.
set -uo pipefail
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/base_r06.so timeout -k 10 300 python tools/scan_bitwise.py dump $O/base.npz > $O/dump_base.txt 2>&1 || { echo "dump base rc $?"; tail -5 $O/dump_base.txt; exit 1; }
timeout -k 10 300 python tools/scan_bitwise.py dump $O/head.npz > $O/dump_head.txt 2>&1 || { echo "dump head rc $?"; tail -5 $O/dump_head.txt; exit 1; }
python tools/scan_bitwise.py compare $O/base.npz $O/head.npz > $O/bitwise.txt 2>&1; tail -3 $O/bitwise.txt
rm -f $O/base.npz $O/head.npz
timeout -k 10 400 python tools/scan_ab_libs.py 4 32:501,32:1501 tools/_variants/base_r06.so velocity-asr_amd/velocity_asr/lib/libvasr_hip.so tools/_variants_scan/lib_0_up4.so tools/_variants_scan/lib_1_up3.so tools/_variants_scan/lib_2_nocache.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
VASR_LIB=tools/_variants/scan_stamps.so timeout -k 10 200 python tools/diag/scan_l_clock.py 4 20 > $O/l_clock.txt 2>&1 || { echo "lclock rc $?"; tail -5 $O/l_clock.txt; exit 1; }
grep -v amdgpu.ids $O/l_clock.txt
