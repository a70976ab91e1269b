#!/bin/bash
# r05ab: upper-stack levels >= 5 in LDS (the 16-step scan at L > 512 back to three waves per SIMD): outputs
# bitwise vs the round-start library, launch times at 30 s (L = 1501) and 10 s, C4 bench lines interleaved.
set -uo pipefail
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/base_r05m.so timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_base.npz > $O/bitwise_base.txt 2>&1 || { echo "dump base rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_base.txt; exit 1; }
timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_head.npz > $O/bitwise_head.txt 2>&1 || { echo "dump head rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_head.txt; exit 1; }
timeout -k 10 120 python -u tools/scan_bitwise.py compare $O/scan_base.npz $O/scan_head.npz > $O/bitwise_compare.txt 2>&1; rm -f $O/*.npz; tail -1 $O/bitwise_compare.txt
for bl in "32 1501" "16 1501" "32 501"; do
set -- $bl
SCAN_MODES=2 SCAN_B=$1 SCAN_L=$2 VARIANT_DIR=_abl9 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/b$1_l$2.txt 2>&1 || { echo "b$1 rc $?"; tail -5 $O/b$1_l$2.txt; exit 1; }
echo "B=$1 L=$2"; cat $O/b$1_l$2.txt
done
for r in 1 2; do
for lib in head_r05 head_up; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --seconds 30 > $O/c4_${lib}_$r.json 2> $O/c4_${lib}_$r.err || { echo "c4 $lib rc $?"; tail -3 $O/c4_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4_${lib}_$r.json')); s=d['config']['schedule']; print('c4 $lib $r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline']['avg_launch_us'], d['machine']['clock_ghz'])"
done
done
