#!/bin/bash
# r06ag: the composed-fusion tests.
set -uo pipefail
O=gpurun_out/r06ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_compose.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -8 $O/tests.txt; exit $rc
