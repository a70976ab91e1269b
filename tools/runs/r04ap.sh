#!/bin/bash
# r04ap: the fused tail's ablations (r04an) and the A-read pipelining (r04ao) graph-timed at
# small M (one utterance's blocks), where r04an's Python-call timing measured the host.
set -uo pipefail
O=gpurun_out/r04ap
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
for v in tailab1 tailab2 tailab4 tailab3 tap2; do
  VASR_LIB=tools/_variants/$v.so run $v timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
done
VASR_TAIL_WAVES=12 run base_w12 timeout -k 10 120 python tools/diag/tail_time.py 501 1024
VASR_TAIL_WAVES=6 run base_w6 timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
VASR_TAIL_ROWS=32 run base_r32 timeout -k 10 120 python tools/diag/tail_time.py 501 1024
cat $O/base.txt $O/tailab1.txt $O/tailab2.txt $O/tailab4.txt $O/tailab3.txt $O/tap2.txt $O/base_w12.txt $O/base_w6.txt $O/base_r32.txt | grep M=
