#!/bin/bash
# r03b: the pruned ABI (v12) + bench-workload goldens: full GPU suite, smoke, the four bench configs.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
export VASR_PARITY_LOG=$O/parity.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
unset VASR_PARITY_LOG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python bench.py --bf16 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python bench.py --int8 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python bench.py --seconds 30 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
echo done > $O/DONE
