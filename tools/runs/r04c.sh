#!/bin/bash
# r04c: the vmcnt fix (scan: vmcnt(0) before the output stores; rows GEMM loaders: vmcnt(0)) --
# interference matrix, probe stress (eager + graphs), the original graph stress, kernel timings
# vs the pre-fix library.
set -uo pipefail
O=gpurun_out/r04c
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run interference timeout -k 10 200 python -u tools/diag/interference.py 30
run probe_eager timeout -k 10 200 python -u tools/diag/graph_probe.py eager 32 4 25
run probe_graph timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
run stress_caller32 timeout -k 10 250 python -u tools/diag/graph_stress.py caller 32
for lib in default pre; do
  if [ $lib = pre ]; then export VASR_LIB=tools/_variants/pre.so; else unset VASR_LIB; fi
  run rows_$lib timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
  run scan32_$lib timeout -k 10 60 python -u tools/scan_bench.py 32 501 384 64 2 50
  run scan16_$lib timeout -k 10 60 python -u tools/scan_bench.py 16 501 384 64 2 50
  run scan32c4_$lib timeout -k 10 60 python -u tools/scan_bench.py 32 1501 384 64 2 20
done
unset VASR_LIB
grep -v "libdrm" $O/interference.txt | awk '$0 !~ / 0\/30/'
grep -h "MODE\|lib=\|^scan" $O/*.txt
