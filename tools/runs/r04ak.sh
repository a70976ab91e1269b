#!/bin/bash
# r04ak: chunked scan with the level composites merged inside the output launch (2 launches instead
# of 3 for nch <= 32): bitwise tests, scan time at B = 1 vs the 3-launch form, B = 1 latency.
set -uo pipefail
O=gpurun_out/r04ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_scan_chunked.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed"; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 100 python -u tools/scan_bench.py 1 501 384 64 2 50 chunked > $O/scan_new$i.txt 2>&1 || exit 1
  VASR_LIB=tools/_variants/nofuse.so timeout -k 10 100 python -u tools/scan_bench.py 1 501 384 64 2 50 chunked > $O/scan_old$i.txt 2>&1 || exit 1
  timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline > $O/b1_new$i.json 2>/dev/null || exit 1
  VASR_LIB=tools/_variants/nofuse.so timeout -k 10 200 python bench.py --inproc --batch 1 --steps 50 --warmup 10 --no-cpu-baseline > $O/b1_old$i.json 2>/dev/null || exit 1
done
for f in $O/scan_*.txt; do echo "$f: $(grep -v libdrm $f | tail -1)"; done
for f in $O/b1_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['tokens_vs_reference']['clips_identical'])"; done
