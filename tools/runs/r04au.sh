#!/bin/bash
# r04au: the pipelined tail's wave counts (4 / 6 / 12 per workgroup) at both row forms, graph-timed.
set -uo pipefail
O=gpurun_out/r04au
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
for w in 12 6 4; do
  VASR_TAIL_WAVES=$w run w$w timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
done
run w12b timeout -k 10 120 python tools/diag/tail_time.py 501 1024 8016 16032
for w in 12 6 4 12b; do sed "s/^/w$w /" $O/w$w.txt | grep M=; done
