#!/bin/bash
# r04x: rows engine with the two waves of a SIMD in opposite phase orders (stagger) vs without,
# cycle stamps of the new form, rows-vs-tiles bitwise, concurrency tests, bench x2.
set -uo pipefail
O=gpurun_out/r04x
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -8 $O/$n.txt; exit $rc; }
}
for i in 1 2; do
  run rows_new$i timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
  VASR_LIB=tools/_variants/nostagger.so run rows_old$i timeout -k 10 120 python -u tools/rows_bench.py 8016 16032
done
VASR_LIB=tools/_variants/rowstamps.so run stamps timeout -k 10 120 python -u tools/diag/rows_stamps.py 8016 16032
run bitwise timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "rows_engine"
run concurrent timeout -k 10 300 python -u -m pytest tests/test_concurrent_gpu.py -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  timeout -k 10 250 python bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
  VASR_LIB=tools/_variants/nostagger.so timeout -k 10 250 python bench.py --no-cpu-baseline > $O/bench_old$i.json 2> $O/bench_old$i.err || { echo "bench old rc $?"; exit 1; }
done
grep -h "M=" $O/rows_*.txt $O/stamps.txt
tail -1 $O/bitwise.txt; tail -1 $O/concurrent.txt
for f in $O/bench*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'], d['roofline']['gemm_avg_launch_us'], d['graph_tokens_match_eager'])"; done
