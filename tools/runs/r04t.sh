#!/bin/bash
# r04t: run-to-run spread of the default bench line on one box (3 x two-group default, 2 x one graph), interleaved.
set -uo pipefail
O=gpurun_out/r04t
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/d$i.json 2> $O/d$i.err || { echo "d$i rc $?"; exit 1; }
  [ $i -le 2 ] && { timeout -k 10 200 python bench.py --no-cpu-baseline --streams 1 > $O/s$i.json 2> $O/s$i.err || { echo "s$i rc $?"; exit 1; }; }
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['graph_tokens_match_eager'])"; done
