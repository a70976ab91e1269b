#!/bin/bash
# r05g: scan outputs bitwise vs the library before the N = 128 scalar pair-sum (tools/scan_bitwise.py,
# 259 cases), the GPU suite, and two default bench lines (per-step device times, clock after the
# timed steps).
set -uo pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/base_r05.so timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_base.npz > $O/bitwise_base.txt 2>&1 || { echo "dump base rc $?"; tail -5 $O/bitwise_base.txt; exit 1; }
timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_head.npz > $O/bitwise_head.txt 2>&1 || { echo "dump head rc $?"; tail -5 $O/bitwise_head.txt; exit 1; }
timeout -k 10 120 python -u tools/scan_bitwise.py compare $O/scan_base.npz $O/scan_head.npz > $O/bitwise_compare.txt 2>&1; tail -3 $O/bitwise_compare.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/proj_width.py > $O/proj_width.txt 2>&1 || { echo "proj rc $?"; exit 1; }
cat $O/proj_width.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$i.json')); print(d['value'], d['ms_per_step'], d['machine'], d['step_ms_device'], d['roofline']['avg_launch_us'], d['config']['schedule']['ms_per_replay_by_streams'])"
done
