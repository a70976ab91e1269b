#!/bin/bash
# r05ag: bench line with the two-group schedule forced (the whole-batch scan launch reported beside the group's).
set -uo pipefail
O=gpurun_out/r05ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 2 > $O/s2.json 2> $O/s2.err || { echo "rc $?"; tail -5 $O/s2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/s2.json')); r=d['roofline']; print(d['value'], r['avg_launch_us'], r['frac'], r.get('whole_batch_launch'))"
