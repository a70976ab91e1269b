#!/bin/bash
# r03ag: 8-wave (32-channel) streaming-scan workgroups for 4 states per lane / 32-step chunks (VASR_SCAN_BW=8):
# bitwise vs 4-wave blocks, scan timing, e2e A/B.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 300 python tools/scan_bitwise.py dump $O/bw4.npz > $O/bitwise.txt 2>&1
VASR_SCAN_BW=8 timeout -k 10 300 python tools/scan_bitwise.py dump $O/bw8.npz >> $O/bitwise.txt 2>&1
timeout -k 10 60 python tools/scan_bitwise.py compare $O/bw4.npz $O/bw8.npz >> $O/bitwise.txt 2>&1
rm -f $O/bw4.npz $O/bw8.npz
for B in 8 16 21; do
  for bw in 4 8; do
    echo "bw=$bw" >> $O/scan.txt
    VASR_SCAN_BW=$bw timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan.txt 2>&1
  done
done
timeout -k 10 900 python tools/ab_matrix.py $O/ab 3 'bw4|VASR_SCAN_BW=4|' 'bw8|VASR_SCAN_BW=8|' > $O/ab.txt 2>&1
VASR_SCAN_BW=8 timeout -k 10 300 python bench.py --seconds 30 --no-cpu-baseline > $O/bench_c4_bw8.json 2> $O/bench_c4_bw8.err
timeout -k 10 300 python bench.py --seconds 30 --no-cpu-baseline > $O/bench_c4_bw4.json 2> $O/bench_c4_bw4.err
echo done > $O/DONE
