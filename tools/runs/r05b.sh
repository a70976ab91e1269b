#!/bin/bash
# r05b: (1) the packed-fp32 SGPR write-after-read hazard alone (tools/ubench/pk_sgpr_war.hip),
# victim alone / beside MFMA chains / beside VALU chains; (2) the GPU suite with the new stress and
# probe tests; (3) the default bench line (machine record, warm-up reference check).
set -uo pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 ./tools/ubench/bin/pk_sgpr_war 20 4000 6000 > $O/pk_sgpr_war.txt 2>&1; rc=$?
echo "rc $rc" >> $O/pk_sgpr_war.txt; cat $O/pk_sgpr_war.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['machine'], d['roofline']['avg_launch_us'], d['config']['schedule'], d['warmup_tokens_vs_reference']['all_ranks_pass'])"
