#!/bin/bash
# r04g: isolate the mode-2 ingredient that goes wrong beside co-resident MFMA kernels: the tree's
# fused multiply-adds, the {dt, x*dt} pre-pass, the packed y partial.
set -uo pipefail
O=gpurun_out/r04g
mkdir -p $O
export ONLY_VICTIMS=scan AGGRESSORS="ssm_block_tail[(1024;gemm[(8016, 192), (384;gemm_argmax"
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run base timeout -k 10 120 python -u tools/diag/interference.py 40
for v in nofma noprep scaly; do
  run $v env VASR_LIB=tools/_variants/$v.so timeout -k 10 120 python -u tools/diag/interference.py 40
done
for f in base nofma noprep scaly; do echo "== $f"; grep "victim" $O/$f.txt; done
