#!/bin/bash
# r04r: the default bench line (two utterance groups, concurrent), the one-graph form for
# comparison, and one line per BASELINE config (tools/config_benches.sh).
set -uo pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench rc $?"; tail -5 $O/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --streams 1 --no-cpu-baseline > $O/bench_s1.json 2> $O/bench_s1.err || { echo "s1 bench rc $?"; tail -5 $O/bench_s1.err; exit 1; }
bash tools/config_benches.sh r04r || { echo "config benches failed"; exit 1; }
cat $O/bench_default.json $O/bench_s1.json
for f in gpurun_out/cfg_r04r/*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d.get('tokens_vs_reference'))")"; done
