#!/bin/bash
# r06ax: XCD-run block order for the front end (STFT, log-mel, norm; VASR_FE_XCD 1 HEAD / 0), stft+mel pair A/B,
# then the front-end parity tests on the HEAD library.
set -uo pipefail
O=gpurun_out/r06ax; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/fe_ab_libs.py 8 32:160000,32:480000,16:160000 $V/fexcd0.so $V/fexcd1.so > $O/fe_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/fe_ab.txt; exit 1; }
cat $O/fe_ab.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_ragged.py > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; exit $rc
