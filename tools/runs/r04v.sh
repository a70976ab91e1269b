#!/bin/bash
# r04v: rows-engine loader waves waiting for a count of their younger LDS-DMA loads instead of
# vmcnt(0): GEMM time at the bench's shapes (A/B/C interleaved x2), rows-vs-tiles bitwise, the
# concurrency tests and the graph probe on the new default.
set -uo pipefail
O=gpurun_out/r04v
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -8 $O/$n.txt; exit $rc; }
}
for i in 1 2; do
  run rows_new$i timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
  VASR_LIB=tools/_variants/lw0.so run rows_lw0_$i timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
  VASR_LIB=tools/_variants/lw1nowait.so run rows_nowait$i timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
done
run bitwise timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "rows_engine"
run concurrent timeout -k 10 300 python -u -m pytest tests/test_concurrent_gpu.py -x -q --timeout 200 --timeout-method thread
run probe timeout -k 10 300 python -u tools/diag/graph_probe.py graph 32 4 50
grep -h "M=\|us" $O/rows_*.txt | grep -v "^rc" | head -40
tail -1 $O/bitwise.txt; tail -1 $O/concurrent.txt; grep MODE $O/probe.txt
