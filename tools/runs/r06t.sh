#!/bin/bash
# r06t: the argmax CTC head (N = 1000, K = 192) on the rows engine with the transposed epilogue vs the tile
# engine (HEAD) vs rows untransposed: keys compared bitwise, interleaved A/B; argmax tests; C2 lines A/B.
set -uo pipefail
O=gpurun_out/r06t; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 6 16032:1000:-1,48032:1000:-1,8016:1000:-1 $V/am_tiles.so $V/am_rows_t.so $V/am_rows_plain.so > $O/argmax_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/argmax_ab.txt; exit 1; }
cat $O/argmax_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_fused_argmax.py tests/test_gpu_parity.py tests/test_int8.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', d['value'], d['ms_per_step'], (d['tokens_vs_reference'] or {}).get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
for r in 1 2; do
for v in am_tiles am_rows_t; do
VASR_LIB=$PWD/$V/$v.so timeout -k 10 300 python bench.py --inproc --no-cpu-baseline > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { echo "bench rc $?"; tail -5 $O/c2_${v}_$r.err; exit 1; }
summ $O/c2_${v}_$r.json c2_${v}_$r
done
done
