#!/bin/bash
# r04ao: the fused tail's A-fragment reads one step ahead of their MFMAs (VASR_TAIL_APIPE) at
# three weight-prefetch depths of the 32-row form, and the shallower prefetch alone; output
# digests must equal the library's.
set -uo pipefail
O=gpurun_out/r04ao
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python tools/diag/tail_time.py 501 8016 16032
for v in tap4 tap3 tap2 tpd2; do
  VASR_LIB=tools/_variants/$v.so run $v timeout -k 10 120 python tools/diag/tail_time.py 501 8016 16032
done
run base2 timeout -k 10 120 python tools/diag/tail_time.py 501 8016 16032
cat $O/base.txt $O/tap4.txt $O/tap3.txt $O/tap2.txt $O/tpd2.txt $O/base2.txt | grep M=
