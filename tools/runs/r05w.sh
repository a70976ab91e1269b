#!/bin/bash
# r05w: round-5 profile at HEAD (scan wave priority): kernel trace + stats of the default bench command,
# FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), SQ counters of the 32- and 16-clip scan launches
# (tools/pmc_kernel.sh), MFMA counters of the composed projection at M = 16032 (tools/pmc_mfma.sh).
set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/profile.sh r05w || { echo "profile rc $?"; exit 1; }
timeout -k 10 700 bash tools/pmc_kernel.sh r05w_scan32 python3 tools/scan_bench.py 32 501 384 64 2 50 || { echo "pmc32 rc $?"; exit 1; }
timeout -k 10 700 bash tools/pmc_kernel.sh r05w_scan16 python3 tools/scan_bench.py 16 501 384 64 2 50 || { echo "pmc16 rc $?"; exit 1; }
timeout -k 10 300 bash tools/pmc_mfma.sh r05w 16032 || { echo "mfma rc $?"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/prof_r05w/bench_trace.json')); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
