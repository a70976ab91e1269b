#!/bin/bash
# r04o: the library with the STFT built without packed-fp32 VALU -- STFT parity, the two-group
# graph probe, the 400-replay caller-stream stress and the concurrency GPU tests.
set -uo pipefail
O=gpurun_out/r04o
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run parity timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stft or mel or fullbatch or c4"
run seq timeout -k 10 200 python -u tools/diag/interference_seq.py 10 20 0,1,2 4 12
run probe_graph timeout -k 10 300 python -u tools/diag/graph_probe.py graph 32 8 50
run stress_caller32 timeout -k 10 250 python -u tools/diag/graph_stress.py caller 32
run concurrent timeout -k 10 300 python -u -m pytest tests/test_concurrent_gpu.py -x -q --timeout 200 --timeout-method thread
tail -2 $O/parity.txt
grep -h aggressor $O/seq.txt
grep -h "MODE\|mismatching replays" $O/*.txt
tail -2 $O/concurrent.txt
