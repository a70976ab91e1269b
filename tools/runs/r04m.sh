#!/bin/bash
# r04m: the pattern of the STFT perturbation (DETAIL), other victims beside the same aggressor
# sequence, and the aggressor GEMM without its MFMAs (VASR_X3_ABLATE=1 variant).
set -uo pipefail
O=gpurun_out/r04m
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
DETAIL=1 run seq_detail timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 1,2,3 0,1,2
VICTIM=3 run vic_ln timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 0,1,2 12
VICTIM=4 run vic_dwconv timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 0,1,2 12
VICTIM=6 run vic_scan timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 0,1,2 12
VASR_LIB=tools/_variants/x3nomfma.so run seq_nomfma timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 1,2,3 0,1,2 12
grep -h "aggressor\|victim:\|workgroups" $O/*.txt
