#!/bin/bash
# r04h: the fix -- mode 2 forms x*dt per lane (no {dt, x*dt} LDS slab) + M0-safe LDS-DMA asm in the
# GEMMs.  Scan outputs bitwise vs the previous library (259 cases), interference matrix, probes,
# the original 400-replay stress, the GPU test suite, bench one graph vs two groups.
set -uo pipefail
O=gpurun_out/r04h
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run bitwise_head env VASR_LIB=tools/_variants/head.so timeout -k 10 200 python -u tools/scan_bitwise.py dump $O/head.npz
run bitwise_new timeout -k 10 200 python -u tools/scan_bitwise.py dump $O/new.npz
run bitwise_cmp timeout -k 10 60 python -u tools/scan_bitwise.py compare $O/head.npz $O/new.npz
rm -f $O/head.npz $O/new.npz
run interference env VICTIMS="ssm_scan[(1024" timeout -k 10 200 python -u tools/diag/interference.py 40
run probe_eager timeout -k 10 200 python -u tools/diag/graph_probe.py eager 32 4 25
run probe_graph timeout -k 10 200 python -u tools/diag/graph_probe.py graph 32 8 25
run stress_caller32 timeout -k 10 250 python -u tools/diag/graph_stress.py caller 32
for lib in new head; do
  if [ $lib = head ]; then export VASR_LIB=tools/_variants/head.so; else unset VASR_LIB; fi
  run scan32_$lib timeout -k 10 60 python -u tools/scan_bench.py 32 501 384 64 2 50
  run scan16_$lib timeout -k 10 60 python -u tools/scan_bench.py 16 501 384 64 2 50
done
unset VASR_LIB
run pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for s in 1 2 1 2; do
  run bench_s$s timeout -k 10 300 python bench.py --inproc --no-cpu-baseline --no-scatter --streams $s
done
tail -3 $O/bitwise_cmp.txt
grep "victim" $O/interference.txt | awk '$0 !~ / 0\/40/'
grep -h "MODE\|^scan" $O/*.txt
tail -2 $O/pytest_gpu.txt
for f in $O/bench_s*.txt; do python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['tokens_vs_reference']['clips_identical'], d['roofline']['avg_launch_us'])"; done
