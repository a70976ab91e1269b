#!/bin/bash
# r05ap: time-split scan, ready flags + wave priorities (phase 1 first).
# three-launch (1) and one-launch (2) forms interleaved, and a kernel trace of the B = 1 line.
set -uo pipefail
O=gpurun_out/r05ap
mkdir -p $O $O/prof_b1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_scan_chunked.py tests/test_host.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 1 2; do
    for sec in 10 30; do
      VASR_SCAN_SPLIT=$sp timeout -k 10 200 python bench.py --inproc --batch 1 --seconds $sec --steps 50 --warmup 10 \
        --no-cpu-baseline --roofline-steps 2 > $O/b1_${sec}s_split${sp}_$rep.json 2> $O/b1_${sec}s_split${sp}_$rep.err || { echo "b1 rc $?"; tail -5 $O/b1_${sec}s_split${sp}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b1_${sec}s_split${sp}_$rep.json')); print('$sec s split $sp', d['value'], d['ms_per_step'], d.get('launches_per_step'), d['roofline']['avg_launch_us'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b1/trace -o run --output-format csv -- python3 bench.py --inproc --batch 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_b1/b1.json 2> $O/prof_b1/b1.err || { echo "b1 prof rc $?"; exit 1; }
echo profile done
VASR_LIB=tools/_variants/split_stamps.so timeout -k 10 120 python tools/diag/split_stamps.py 501 20 > $O/stamps501.txt 2>&1 && VASR_LIB=tools/_variants/split_stamps.so timeout -k 10 120 python tools/diag/split_stamps.py 1501 20 > $O/stamps1501.txt 2>&1; cat $O/stamps*.txt
