#!/bin/bash
# r04f: which part of the local scan goes wrong beside co-resident MFMA kernels -- the victim scan
# in other forms (mode 0 without the {dt, x*dt} pre-pass, 16-step chunks, 2 states per lane),
# generic butterfly exchanges, a block barrier after the pre-pass.
set -uo pipefail
O=gpurun_out/r04f
mkdir -p $O
export ONLY_VICTIMS=scan AGGRESSORS="ssm_block_tail[(1024;gemm[(8016, 192), (384;gemm_argmax"
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python -u tools/diag/interference.py 40
run mode0 env VASR_SCAN_FMA=0 timeout -k 10 120 python -u tools/diag/interference.py 40
run t16 env VASR_SCAN_T=16 timeout -k 10 120 python -u tools/diag/interference.py 40
run npl2 env VASR_SCAN_NPL=2 timeout -k 10 120 python -u tools/diag/interference.py 40
run xgen env VASR_LIB=tools/_variants/xgen.so timeout -k 10 120 python -u tools/diag/interference.py 40
run prepsync env VASR_LIB=tools/_variants/prepsync.so timeout -k 10 120 python -u tools/diag/interference.py 40
for f in base mode0 t16 npl2 xgen prepsync; do echo "== $f"; grep "victim" $O/$f.txt; done
