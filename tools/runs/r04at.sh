#!/bin/bash
# r04at: rows engine with W fragments two k-steps ahead of their MFMAs (VASR_ROWS_LEAD=2) vs one.
set -uo pipefail
O=gpurun_out/r04at
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
for i in 1 2; do
  run base$i timeout -k 10 120 python tools/rows_bench.py 501 8016 16032
  VASR_LIB=tools/_variants/rl2.so run rl2_$i timeout -k 10 120 python tools/rows_bench.py 501 8016 16032
done
cat $O/base1.txt $O/rl2_1.txt $O/base2.txt $O/rl2_2.txt | grep M=
