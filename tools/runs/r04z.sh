#!/bin/bash
# r04z: cooperative small-M SSM tail -- its tests, the model-level parity suite, B=1 latency and
# its timeline, and the default bench (two-group / one-graph autotuned).
set -uo pipefail
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run tail_tests timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -x -v --timeout 120 --timeout-method thread
run parity timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fwd or forward or token or b1 or pinned"
run b1 timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline
run b1_30 timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 30 --steps 50 --warmup 10 --no-cpu-baseline
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/tl.out 2>&1 || { echo "timeline rc $?"; exit 1; }
python tools/graph_copies.py --summary $O/tl/run_kernel_trace.csv > $O/b1_10s_timeline.txt
run c2 timeout -k 10 250 python bench.py --no-cpu-baseline
grep -E "passed|failed" $O/tail_tests.txt $O/parity.txt | tail -3
for f in b1 b1_30 c2; do python -c "import json; d=json.loads(open('$O/$f.txt').read().splitlines()[-2]); print('$f', d['value'], d['ms_per_step'], d['tokens_vs_reference']['clips_identical'] if d['tokens_vs_reference'] else None, d['graph_tokens_match_eager'])"; done
tail -1 $O/b1_10s_timeline.txt; grep ssm_tail $O/b1_10s_timeline.txt
