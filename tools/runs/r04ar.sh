#!/bin/bash
# r04ar: the tail with A-fragment reads pipelined and 12 waves at 16 rows as the library default:
# tail and model-parity tests, graph-timed tail, B = 1 latency (10 s / 30 s), C2 and C3 benches.
set -uo pipefail
O=gpurun_out/r04ar
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run tail_tests timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py tests/test_concurrent_gpu.py -x -v --timeout 120 --timeout-method thread
run parity timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
run tail_time timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
run b1 timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline
run b1_30 timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 30 --steps 50 --warmup 10 --no-cpu-baseline
run c2 timeout -k 10 250 python bench.py --no-cpu-baseline
run c3 timeout -k 10 250 python bench.py --bf16 --no-cpu-baseline
run c2b timeout -k 10 250 python bench.py --no-cpu-baseline
grep -hE "passed|failed" $O/tail_tests.txt $O/parity.txt | tail -3
grep M= $O/tail_time.txt
for f in b1 b1_30 c2 c3 c2b; do python -c "import json; d=json.loads(open('$O/$f.txt').read().splitlines()[-2]); print('$f', d['value'], d['ms_per_step'], d['tokens_vs_reference']['clips_identical'] if d['tokens_vs_reference'] else None, d['graph_tokens_match_eager'], d['config'].get('schedule', {}).get('ms_per_replay_by_streams'))"; done
