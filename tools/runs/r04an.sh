#!/bin/bash
# r04an: what bounds the fused SSMBlock tail -- ablation builds (no weight loads / no MFMAs /
# no A-fragment LDS reads / no loads and no MFMAs) timed against the library at four M.
set -uo pipefail
O=gpurun_out/r04an
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python tools/diag/tail_time.py
for v in 1 2 4 3; do
  VASR_LIB=tools/_variants/tailab$v.so run ab$v timeout -k 10 120 python tools/diag/tail_time.py
done
run base2 timeout -k 10 120 python tools/diag/tail_time.py
cat $O/base.txt $O/ab1.txt $O/ab2.txt $O/ab4.txt $O/ab3.txt $O/base2.txt | grep M=
