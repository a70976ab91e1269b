#!/bin/bash
# r03ai: HEAD evidence after the caller-stream replay of group 0 (e453602) -- GPU suite, smoke, every
# BASELINE config's bench line, one-utterance latency, rocprofv3 stats + HBM traffic of the C2 bench,
# and a kernel trace of 10 graphed C2 steps (32 x 10 s, 2 groups) for the step's critical path.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ai
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
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/c2 -o run --output-format csv -- python3 tools/graph_copies.py 32 160000 2 > $O/c2.out 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2b.json 2> $O/bench_c2b.err
bash tools/profile.sh r03ai
echo done > $O/DONE
