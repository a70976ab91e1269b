#!/bin/bash
# r05t: scan wave-priority policy (default VASR_SCAN_PRIO=4): outputs bitwise vs the round-start library, the
# policy variants' launch times at B=32 / 16, the GPU suite, default bench lines.
set -uo pipefail
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/base_r05m.so timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_base.npz > $O/bitwise_base.txt 2>&1 || { echo "dump base rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_base.txt; exit 1; }
timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_head.npz > $O/bitwise_head.txt 2>&1 || { echo "dump head rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_head.txt; exit 1; }
timeout -k 10 120 python -u tools/scan_bitwise.py compare $O/scan_base.npz $O/scan_head.npz > $O/bitwise_compare.txt 2>&1; rm -f $O/*.npz; tail -1 $O/bitwise_compare.txt
for b in 32 16; do
SCAN_MODES=2 SCAN_B=$b VARIANT_DIR=_abl8 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$b.txt 2>&1 || { echo "b$b rc $?"; tail -5 $O/b$b.txt; exit 1; }
cat $O/b$b.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench$i.json')); print(d['value'], d['ms_per_step'], d['machine'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['config']['schedule']['ms_per_replay_by_streams'])"
done
