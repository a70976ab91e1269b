#!/bin/bash
# r06bi: LayerNorm + pool fold on by default: the fold tests, then C2 / C3 lines with VASR_POOL_PRENORM=1 / 0
# interleaved, three rounds of C2.
set -uo pipefail
O=gpurun_out/r06bi; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ln_pair.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 1 0; do
    VASR_POOL_PRENORM=$v timeout -k 10 300 python -u bench.py --inproc --no-cpu-baseline > $O/c2_p${v}_$r.json 2> $O/c2_p${v}_$r.err || { echo "c2 rc $?"; tail -5 $O/c2_p${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_p${v}_$r.json')); print('c2 pool_prenorm=$v', d['value'], d['ms_per_step'])"
  done
done
for v in 1 0; do
  VASR_POOL_PRENORM=$v timeout -k 10 300 python -u bench.py --inproc --no-cpu-baseline --bf16 > $O/c3_p$v.json 2> $O/c3_p$v.err || { echo "c3 rc $?"; tail -5 $O/c3_p$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_p$v.json')); print('c3 pool_prenorm=$v', d['value'], d['ms_per_step'])"
done
