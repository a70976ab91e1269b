#!/bin/bash
# r05o: scan staging by buffer loads + three chunk buffers (one barrier per chunk): outputs bitwise vs the
# round-start library (tools/scan_bitwise.py, 259 cases), scan GPU tests, timing of the variants.
set -uo pipefail
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/base_r05m.so timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_base.npz > $O/bitwise_base.txt 2>&1 || { echo "dump base rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_base.txt; exit 1; }
timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_head.npz > $O/bitwise_head.txt 2>&1 || { echo "dump head rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_head.txt; exit 1; }
timeout -k 10 120 python -u tools/scan_bitwise.py compare $O/scan_base.npz $O/scan_head.npz > $O/bitwise_compare.txt 2>&1; rm -f $O/*.npz; tail -3 $O/bitwise_compare.txt
rm -f $O/*.npz
for b in 32 16; do
SCAN_MODES=2 SCAN_B=$b VARIANT_DIR=_abl7 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$b.txt 2>&1 || { echo "b$b rc $?"; tail -5 $O/b$b.txt; exit 1; }
cat $O/b$b.txt
done
timeout -k 10 600 python -u -m pytest tests/test_scan_chunked.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "scan or mamba or statedim" > $O/scan_tests.txt 2>&1; rc=$?
tail -2 $O/scan_tests.txt; exit $rc
