#!/bin/bash
# r06bh: LayerNorm + adaptive pool fused kernel geometry (HEAD = 8-row groups with per-row branches, 4 waves per
# workgroup; g4w1 / g4w4 / g8w4 unbranched), graph-timed against the two launches, libraries in turn x2.
set -uo pipefail
O=gpurun_out/r06bh; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
for r in 1 2; do
  for l in lp_head lp_g4w1 lp_g4w4 lp_g8w4; do
    VASR_LIB=$V/$l.so timeout -k 10 120 python -u tools/lnpool_bench.py 32:64:16,32:188:46,1:64:16 >> $O/lnpool.txt 2>&1 || { echo "rc $? $l"; tail -5 $O/lnpool.txt; exit 1; }
  done
done
cat $O/lnpool.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_ln_pair.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; exit $rc
