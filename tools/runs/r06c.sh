#!/bin/bash
# r06c: z-in-tail after the contraction fix: bitwise tests, diagnostics, C2 bench A/B (z-in-tail on / off).
set -uo pipefail
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ssm_tail.py -x -q --timeout 120 --timeout-method thread > $O/tail_tests.txt 2>&1; rc=$?
tail -3 $O/tail_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/diag/zt_diag.py 32 501 > $O/diag_32.txt 2>&1 || { echo "diag rc $?"; tail -20 $O/diag_32.txt; exit 1; }
grep -v amdgpu.ids $O/diag_32.txt
for r in 1 2; do
for z in 1 0; do
VASR_Z_IN_TAIL=$z timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_z${z}_$r.json 2> $O/c2_z${z}_$r.err || { echo "bench rc $?"; tail -5 $O/c2_z${z}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2_z${z}_$r.json')); s=d['config']['schedule']; print('c2 z$z $r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['kernels']['ssm_tail_isolated_us'], d['roofline']['gemm_avg_launch_us'], d['tokens_vs_reference']['all_ranks_pass'], d['machine']['clock_ghz'])"
done
done
