#!/bin/bash
# r04k: after draining the tile GEMM's untracked LDS-DMA before its epilogue / exit -- prefixes of
# group 0's pipeline beside group 1's STFT launches, the graph probe, the 400-replay stress, the
# concurrency GPU tests.
set -uo pipefail
O=gpurun_out/r04k
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run seq timeout -k 10 300 python -u tools/diag/interference_seq.py 10 10
run probe_graph timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
run stress_caller32 timeout -k 10 250 python -u tools/diag/graph_stress.py caller 32
run concurrent timeout -k 10 300 python -u -m pytest tests/test_concurrent_gpu.py -x -q --timeout 200 --timeout-method thread
grep -v libdrm $O/seq.txt | grep aggressor
grep -h "MODE" $O/*.txt
tail -2 $O/concurrent.txt
