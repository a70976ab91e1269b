#!/bin/bash
# r04aq: A-read pipelining (VASR_TAIL_APIPE) with the 32-row prefetch at 2 steps and the 16-row
# 12-wave form's at 5 / 4, against the library, 4 and 12 waves at 16 rows; graph-timed.
set -uo pipefail
O=gpurun_out/r04aq
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
VASR_TAIL_WAVES=12 run base_w12 timeout -k 10 120 python tools/diag/tail_time.py 501 1024
VASR_LIB=tools/_variants/tapA.so run tapA timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
VASR_LIB=tools/_variants/tapA.so VASR_TAIL_WAVES=12 run tapA_w12 timeout -k 10 120 python tools/diag/tail_time.py 501 1024
VASR_LIB=tools/_variants/tapB.so VASR_TAIL_WAVES=12 run tapB_w12 timeout -k 10 120 python tools/diag/tail_time.py 501 1024
run base2 timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
cat $O/base.txt $O/base_w12.txt $O/tapA.txt $O/tapA_w12.txt $O/tapB_w12.txt $O/base2.txt | grep M=
