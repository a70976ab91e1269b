#!/bin/bash
# r04e: where the local scan's corrupted outputs sit (clip, step, channel) under a co-resident aggressor
set -uo pipefail
O=gpurun_out/r04e
mkdir -p $O
DETAIL=1 ONLY_VICTIMS=scan timeout -k 10 200 python -u tools/diag/interference.py 40 > $O/detail.txt 2>&1; rc=$?
echo "rc $rc" >> $O/detail.txt
grep -v "libdrm\| 0/40" $O/detail.txt | head -150
exit $rc
