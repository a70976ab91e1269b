#!/bin/bash
# r04am: the fused SSMBlock tail with fp32 weight fragments split in registers (4 B per weight)
# vs pre-split bf16 planes (6 B): tail tests, isolated timing at three prefetch settings, B = 1
# latency and the default bench.
set -uo pipefail
O=gpurun_out/r04am
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run tail_tests timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -x -v --timeout 120 --timeout-method thread
run tw_default timeout -k 10 120 python tools/diag/tail_weights.py
VASR_LIB=tools/_variants/tailpd31.so run tw_pd31 timeout -k 10 120 python tools/diag/tail_weights.py
VASR_LIB=tools/_variants/tailpd63.so run tw_pd63 timeout -k 10 120 python tools/diag/tail_weights.py
run b1 timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline
VASR_TAIL_WEIGHTS=planes run b1_planes timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline
run c2 timeout -k 10 250 python bench.py --no-cpu-baseline
VASR_TAIL_WEIGHTS=planes run c2_planes timeout -k 10 250 python bench.py --no-cpu-baseline
grep -E "passed|failed" $O/tail_tests.txt | tail -2
cat $O/tw_default.txt $O/tw_pd31.txt $O/tw_pd63.txt | grep M=
for f in b1 b1_planes c2 c2_planes; do python -c "import json; d=json.loads(open('$O/$f.txt').read().splitlines()[-2]); print('$f', d['value'], d['ms_per_step'], d['tokens_vs_reference']['clips_identical'] if d['tokens_vs_reference'] else None, d['graph_tokens_match_eager'], d['config'].get('schedule'))"; done
