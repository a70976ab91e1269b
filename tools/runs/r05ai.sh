#!/bin/bash
# r05ai: rows engine with wide C stores (in-register quad transposes, 4 dwordx4 per chunk) vs the dword form:
# bitwise test vs the tile engine, projection launch times, C2 one-graph bench lines interleaved.
set -uo pipefail
O=gpurun_out/r05ai
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rows_engine" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for lib in head_narrow head_wide head_narrow head_wide; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 200 python -u tools/diag/proj_width.py > $O/pw_$lib.txt 2>&1 || { echo "pw rc $?"; tail -3 $O/pw_$lib.txt; exit 1; }
echo "$lib $(grep 'N=1280' $O/pw_$lib.txt)"
done
for r in 1 2; do
for lib in head_narrow head_wide; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 1 > $O/c2_${lib}_$r.json 2> $O/c2_${lib}_$r.err || { echo "c2 $lib rc $?"; tail -3 $O/c2_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2_${lib}_$r.json')); r=d['roofline']; print('c2 $lib $r', d['value'], d['ms_per_step'], r.get('gemm_avg_launch_us'), r.get('gemm_insitu_avg_launch_us'), d['machine']['clock_ghz'])"
done
done
