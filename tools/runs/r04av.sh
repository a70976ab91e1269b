#!/bin/bash
# r04av: the pipelined tail's 16-row forms at large M (two 4-wave blocks per CU, or one 12-wave)
# against the 32-row 12-wave default, graph-timed.
set -uo pipefail
O=gpurun_out/r04av
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python tools/diag/tail_time.py 4097 8016 16032
VASR_TAIL_ROWS=16 VASR_TAIL_WAVES=4 run r16w4 timeout -k 10 120 python tools/diag/tail_time.py 4097 8016 16032
VASR_TAIL_ROWS=16 VASR_TAIL_WAVES=12 run r16w12 timeout -k 10 120 python tools/diag/tail_time.py 4097 8016 16032
VASR_TAIL_ROWS=16 VASR_TAIL_WAVES=6 run r16w6 timeout -k 10 120 python tools/diag/tail_time.py 4097 8016 16032
run base2 timeout -k 10 120 python tools/diag/tail_time.py 4097 8016 16032
for n in base r16w4 r16w12 r16w6 base2; do sed "s/^/$n /" $O/$n.txt | grep M=; done
