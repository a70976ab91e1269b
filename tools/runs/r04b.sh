#!/bin/bash
# r04b: interference matrix -- which concurrently running kernel corrupts the STFT / scan output
set -uo pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python -u tools/diag/interference.py 30 > $O/interference.txt 2>&1; rc=$?
echo "rc $rc" >> $O/interference.txt
grep -v "libdrm" $O/interference.txt | awk '$0 !~ / 0\/30/' | head -80
exit $rc
