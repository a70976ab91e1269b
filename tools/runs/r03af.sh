#!/bin/bash
# r03af: HEAD evidence -- GPU suite, smoke, every BASELINE config's bench line, one-utterance latency (10 s, 30 s),
# rocprofv3 kernel stats + HBM traffic of the C2 bench, scan SQ counters at the 16-clip launch.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
export VASR_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
unset VASR_PARITY_LOG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python bench.py --bf16 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python bench.py --seconds 30 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python bench.py --int8 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/bench_b1_10s.json 2> $O/bench_b1_10s.err
timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 30 --steps 30 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/bench_b1_30s.json 2> $O/bench_b1_30s.err
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/b1 -o run --output-format csv -- python3 tools/graph_copies.py 1 160000 1 > $O/b1.out 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2b.json 2> $O/bench_c2b.err
bash tools/profile.sh r03af
VASR_SCAN_NPL=4 VASR_SCAN_T=32 bash tools/pmc_kernel.sh r03af_scan python3 tools/scan_bench.py 16 501 384 64 2 20
echo done > $O/DONE
