#!/bin/bash
# r05aq: time-split scan auto rule (L <= 512) and its use for short L (global blocks at B = 1):
# full GPU suite, then one-utterance latency A/B interleaved:
#   A = three launches, short L streaming (round-start behaviour); B = defaults; C = split for L > 160 only.
set -uo pipefail
O=gpurun_out/r05aq
mkdir -p $O $O/prof_b1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
run() {  # tag sec env...
  local tag=$1 sec=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --inproc --batch 1 --seconds $sec --steps 50 --warmup 10 \
    --no-cpu-baseline --roofline-steps 2 > $O/b1_${sec}s_${tag}.json 2> $O/b1_${sec}s_${tag}.err || { echo "b1 rc $?"; tail -5 $O/b1_${sec}s_${tag}.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b1_${sec}s_${tag}.json')); print('$sec s $tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2 3; do
  run A$rep 10 VASR_SCAN_SPLIT=1 VASR_SCAN_SPLIT_SHORT=0 || exit 1
  run B$rep 10 VASR_SCAN_SPLIT=0 || exit 1
  run C$rep 10 VASR_SCAN_SPLIT_SHORT=0 || exit 1
done
run A1 30 VASR_SCAN_SPLIT=1 VASR_SCAN_SPLIT_SHORT=0 || exit 1
run B1 30 VASR_SCAN_SPLIT=0 || exit 1
run A2 30 VASR_SCAN_SPLIT=1 VASR_SCAN_SPLIT_SHORT=0 || exit 1
run B2 30 VASR_SCAN_SPLIT=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b1/trace -o run --output-format csv -- python3 bench.py --inproc --batch 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_b1/b1.json 2> $O/prof_b1/b1.err || { echo "b1 prof rc $?"; exit 1; }
echo profile done
