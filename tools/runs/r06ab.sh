#!/bin/bash
# r06ab: where one 10-s utterance's 0.56 ms goes: rocprofv3 kernel trace of the batch-1 bench.
set -uo pipefail
O=gpurun_out/r06ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --inproc --no-cpu-baseline --batch 1 --steps 50 --warmup 10 > $O/b1.json 2> $O/b1.err || { echo "rc $?"; tail -5 $O/b1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b1.json')); print(d['value'], d['ms_per_step'])"
