#!/bin/bash
# r04ag: rows engine writing C from the transposed tile (four 16-B stores per chunk): bitwise vs the
# tile engine, GEMM time vs the untransposed form (interleaved x2), parity suite, bench x2 each.
set -uo pipefail
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "rows_engine" > $O/bitwise.txt 2>&1 || { echo "bitwise failed"; tail -20 $O/bitwise.txt; exit 1; }
tail -1 $O/bitwise.txt
for i in 1 2; do
  timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/rows_new$i.txt 2>&1 || exit 1
  VASR_LIB=tools/_variants/notr.so timeout -k 10 100 python -u tools/rows_bench.py 8016 16032 > $O/rows_old$i.txt 2>&1 || exit 1
done
grep -h "M=" $O/rows_*.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -20 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --inproc > $O/bench_new$i.json 2> $O/bn$i.err || exit 1
  VASR_LIB=tools/_variants/notr.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --inproc > $O/bench_old$i.json 2> $O/bo$i.err || exit 1
done
for f in $O/bench_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'], d['config']['schedule']['ms_per_replay_by_streams'], d['roofline']['gemm_avg_launch_us'], d['tokens_vs_reference']['clips_identical'])"; done
