#!/bin/bash
# r03m: fused tail workgroup forms (rows x waves) isolated + B = 1 graph timelines per form
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
timeout -k 10 180 python tools/tail_bench.py 501 1002 4008 8016 > $O/tail.txt 2>&1
for w in 4 6 12; do
  VASR_TAIL_WAVES=$w timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1_w$w -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/b1_w$w.out 2>&1
  VASR_TAIL_WAVES=$w timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/bench_b1_w$w.json 2> $O/bench_b1_w$w.err
done
echo done > $O/DONE
