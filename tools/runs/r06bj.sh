#!/bin/bash
# r06bj: collapse_keys with coalesced row maxima (ck_new, 1024 threads) vs HEAD (ck_head), then the decode tests.
set -uo pipefail
O=gpurun_out/r06bj; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
for r in 1 2; do
  for l in ck_head ck_new; do
    VASR_LIB=$V/$l.so timeout -k 10 120 python -u tools/collapse_bench.py 32:501,32:1501,1:501 >> $O/collapse.txt 2>&1 || { echo "rc $? $l"; tail -5 $O/collapse.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/collapse.txt
timeout -k 10 400 python -u -m pytest tests/test_fused_argmax.py tests/test_ragged.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; exit $rc
