#!/bin/bash
# r04a: locate the concurrent utterance-group race -- first differing kernel output per replay
# (graph caller-stream, eager two streams, graph without packet capture).
set -uo pipefail
O=gpurun_out/r04a
mkdir -p $O
run() {  # run NAME CMD...: stop the script on the first failing GPU step
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run probe_graph timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
run rows_default timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
run rows_loaders2 env VASR_LIB=tools/_variants/loaders2.so timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
run probe_eager timeout -k 10 200 python -u tools/diag/graph_probe.py eager 32 4 25
run probe_graph_nopc env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
run probe_graph_ntoff env VASR_LIB=tools/_variants/ntoff.so timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
grep -h "MODE\|probe span\|lib=" $O/*.txt
