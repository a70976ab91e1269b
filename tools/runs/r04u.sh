#!/bin/bash
# r04u: the autotuned schedule (bench default) x3 and its GPU test, one box.
set -uo pipefail
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_concurrent_gpu.py -x -q --timeout 150 --timeout-method thread > $O/test.txt 2>&1 || { echo "test rc $?"; tail -20 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2 3; do
  timeout -k 10 250 python bench.py --no-cpu-baseline > $O/d$i.json 2> $O/d$i.err || { echo "d$i rc $?"; tail -5 $O/d$i.err; exit 1; }
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['schedule'], d['graph_tokens_match_eager'], d['tokens_vs_reference']['clips_identical'])"; done
