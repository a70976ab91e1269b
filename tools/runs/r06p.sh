#!/bin/bash
# r06p: rows-engine projection with the two waves of a SIMD staggered (store-first loader, MFMA-first
# store-only wave) vs HEAD: bitwise check + interleaved A/B at the bench's projection shapes.
set -uo pipefail
O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 6 16032:896:512,48032:896:512,16032:1280:896,8016:896:512 $V/rows_stag0.so $V/rows_stag1.so > $O/stagger_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/stagger_ab.txt; exit 1; }
cat $O/stagger_ab.txt
