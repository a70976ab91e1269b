#!/bin/bash
# r05ar: argmax keys + CTC collapse in one launch (vasr_ctc_collapse_keys): full GPU suite, then
# interleaved A/B (VASR_COLLAPSE_KEYS=0 two launches vs default one) at B = 1 10 s and at C2.
set -uo pipefail
O=gpurun_out/r05ar
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for ck in 0 1; do
    VASR_COLLAPSE_KEYS=$ck timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 \
      --no-cpu-baseline --roofline-steps 2 > $O/b1_ck${ck}_$rep.json 2> $O/b1_ck${ck}_$rep.err || { echo "b1 rc $?"; tail -5 $O/b1_ck${ck}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b1_ck${ck}_$rep.json')); print('b1 ck$ck', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for ck in 0 1; do
    VASR_COLLAPSE_KEYS=$ck timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_ck${ck}_$rep.json 2> $O/c2_ck${ck}_$rep.err || { echo "c2 rc $?"; tail -5 $O/c2_ck${ck}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_ck${ck}_$rep.json')); print('c2 ck$ck', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'])"
  done
done
