#!/bin/bash
# r05u: chunk-parallel scan (B = 1, 2 at L = 501) with and without the falling wave priority; outputs bitwise.
set -uo pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
for b in 1 2; do
SCAN_FORM=chunked SCAN_MODES=2 SCAN_B=$b VARIANT_DIR=_abl8 timeout -k 10 300 python -u tools/scan_ablate_run.py > $O/ch_b$b.txt 2>&1 || { echo "b$b rc $?"; tail -5 $O/ch_b$b.txt; exit 1; }
cat $O/ch_b$b.txt
done
VASR_LIB=tools/_variants/base_r05m.so timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_base.npz > $O/bitwise_base.txt 2>&1 || { echo "dump base rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_base.txt; exit 1; }
timeout -k 10 300 python -u tools/scan_bitwise.py dump $O/scan_head.npz > $O/bitwise_head.txt 2>&1 || { echo "dump head rc $?"; rm -f $O/*.npz; tail -5 $O/bitwise_head.txt; exit 1; }
timeout -k 10 120 python -u tools/scan_bitwise.py compare $O/scan_base.npz $O/scan_head.npz > $O/bitwise_compare.txt 2>&1; rm -f $O/*.npz; tail -1 $O/bitwise_compare.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch 1 --steps 50 --warmup 10 > $O/b1.json 2> $O/b1.err || { echo "b1 rc $?"; tail -5 $O/b1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b1.json')); print('B=1', d['value'], d['ms_per_step'])"
