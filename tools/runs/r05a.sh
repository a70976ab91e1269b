#!/bin/bash
# r05a: the scan's two launch-time modes.  Default bench line at HEAD, then
# isolated 32-clip scan bursts over time under one PMC pass (clock: GRBM_GUI_ACTIVE / 8 / duration;
# placement: TCC hit rate), the bench again, the bursts again, and bursts without the profiler.
set -uo pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || { echo "bench1 rc $?"; tail -5 $O/bench1.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d $O/pmc1 -o run --output-format csv -- python3 tools/diag/scan_modes.py 25 0.3 10 > $O/modes1.txt 2>&1 || { echo "pmc1 rc $?"; tail -5 $O/modes1.txt; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || { echo "bench2 rc $?"; tail -5 $O/bench2.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P -d $O/pmc2 -o run --output-format csv -- python3 tools/diag/scan_modes.py 25 0.3 10 > $O/modes2.txt 2>&1 || { echo "pmc2 rc $?"; tail -5 $O/modes2.txt; exit 1; }
timeout -k 10 120 python3 tools/diag/scan_modes.py 25 0.3 10 > $O/modes3.txt 2>&1 || { echo "modes3 rc $?"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench3.json 2> $O/bench3.err || { echo "bench3 rc $?"; exit 1; }
for f in $O/bench*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'], d['roofline']['avg_launch_us'])"; done
grep -h scan $O/modes*.txt | awk '{print $4}' | sort -n | uniq -c | head -40
