#!/bin/bash
# r03n: tail 32 rows x 12 waves at M > 4096, rows engine only at M >= 4096: e2e A/B + B = 1
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
timeout -k 10 900 python tools/ab_matrix.py $O/ab 3 'tail4|VASR_TAIL_WAVES=4|' 'auto||' > $O/ab.txt 2>&1
timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/bench_b1.json 2> $O/bench_b1.err
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1 -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/b1.out 2>&1
echo done > $O/DONE
