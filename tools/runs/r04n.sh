#!/bin/bash
# r04n: the STFT built without SLP vectorisation (no packed-fp32 VALU) beside the aggressor
# sequences that perturb the packed build (r04l/r04m).
set -uo pipefail
O=gpurun_out/r04n
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
VASR_LIB=tools/_variants/stftnoslp.so DETAIL=1 run seq_noslp timeout -k 10 300 python -u tools/diag/interference_seq.py 10 20 0,1,2 1,2,3 12 4
run seq_head timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 0,1,2
grep -h "aggressor\|workgroups" $O/*.txt
