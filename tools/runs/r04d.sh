#!/bin/bash
# r04d: interference with more victims (scan, global scan, global tail, tile GEMM), and the scan
# victim with every butterfly exchange through compiler-managed select + dpp_mov / ds_swizzle.
set -uo pipefail
O=gpurun_out/r04d
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run interf_more env VICTIMS="ssm_scan[(1024;ssm_block_tail[(1024;gemm[(8016, 192), (384" ONLY_VICTIMS="ssm_scan;ssm_block_tail;gemm" timeout -k 10 200 python -u tools/diag/interference.py 30
run interf_xgen env VASR_LIB=tools/_variants/xgen.so ONLY_VICTIMS=scan timeout -k 10 200 python -u tools/diag/interference.py 30
for f in interf_more interf_xgen; do echo "== $f"; grep victim $O/$f.txt | awk '$0 !~ / 0\/30/'; done
