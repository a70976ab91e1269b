#!/bin/bash
# r04g: isolate the mode-2 ingredient that goes wrong beside co-resident MFMA kernels: the tree's
# fused multiply-adds, the {dt, x*dt} pre-pass, the packed y partial, wait states after v_exp;
# base = the library with the M0 save / s_nop / restore in the GEMMs' LDS-DMA asm (variants predate it).
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
for v in nofma noprep scaly expnop; do
  run $v env VASR_LIB=tools/_variants/$v.so timeout -k 10 120 python -u tools/diag/interference.py 40
done
run probe_eager timeout -k 10 200 python -u tools/diag/graph_probe.py eager 32 4 25
run probe_graph timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
for v in default rows_nowait rows_d3; do
  if [ $v = default ]; then unset VASR_LIB; else export VASR_LIB=tools/_variants/$v.so; fi
  run rows_$v timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
done
unset VASR_LIB
grep -h "lib=" $O/rows_*.txt
for f in base nofma noprep scaly expnop; do echo "== $f"; grep "victim" $O/$f.txt; done
grep -h MODE $O/probe_*.txt
