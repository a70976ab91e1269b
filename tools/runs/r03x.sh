#!/bin/bash
# r03x: HEAD check after the container restore (GPU suite, smoke, C2 bench) and the scan lane layouts at the
# bench's 16-clip launch: 4 states per lane with 32-step chunks (default) vs 2 per lane with 16 / 32-step chunks,
# alone and end to end.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
for B in 16 32; do
  for v in "4 32" "4 16" "2 16" "2 32"; do
    set -- $v
    echo "npl=$1 T=$2" >> $O/scan.txt
    VASR_SCAN_NPL=$1 VASR_SCAN_T=$2 timeout -k 10 60 python tools/scan_bench.py $B 501 384 64 2 50 >> $O/scan.txt 2>&1
  done
done
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 600 python tools/ab_matrix.py $O/ab 2 'default||' 'npl2t32|VASR_SCAN_NPL=2 VASR_SCAN_T=32|' 'npl2t16|VASR_SCAN_NPL=2 VASR_SCAN_T=16|' > $O/ab.txt 2>&1
echo done > $O/DONE
