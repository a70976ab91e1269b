#!/bin/bash
# r03aj: norm-into-tail + conv-into-GEMM fusion of the local SSM stack: bitwise tests, then
# interleaved end-to-end A/B (VASR_LN_FUSE=1 vs 0) on C2, C5 and C4, then the whole GPU suite.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ln_fuse.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ln_fuse.txt 2>&1
ab() {  # tag, env value, bench args
  VASR_LN_FUSE=$2 timeout -k 10 240 python bench.py --no-cpu-baseline ${@:3} > $O/ab_$1_$2_$i.json 2> $O/ab_$1_$2_$i.err
  python3 - "$O/ab_$1_$2_$i.json" "$1" "$2" >> $O/ab.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d.get("tokens_vs_reference") or {}
print(sys.argv[2], "LN_FUSE=" + sys.argv[3], round(d["value"]), d["ms_per_step"], "tokens", t.get("clips_identical", t.get("pass")))
PY
}
for i in 0 1 2; do ab c2 1; ab c2 0; done
for i in 0; do ab c5 1 --int8; ab c5 0 --int8; ab c4 1 --seconds 30; ab c4 0 --seconds 30; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --inproc --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
echo done > $O/DONE
