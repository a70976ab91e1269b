#!/bin/bash
# r04q: the full GPU test suite and smoke() on the race-fixed library (two-group default).
set -uo pipefail
O=gpurun_out/r04q
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run gpu_tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
grep -E "passed|failed" $O/gpu_tests.txt | tail -2
tail -2 $O/smoke.txt
