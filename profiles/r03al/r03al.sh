#!/bin/bash
# r03al: rows-engine C stores as 16-B-per-lane row segments through a per-wave LDS tile
# (VASR_ROWS_VST=1, default) vs dword stores (0): interleaved end-to-end A/B, GPU suite (no -x), kernel stats.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
ab() {  # tag, env value, bench args
  VASR_ROWS_VST=$2 timeout -k 10 240 python bench.py --no-cpu-baseline ${@:3} > $O/ab_$1_$2_$i.json 2> $O/ab_$1_$2_$i.err
  python3 - "$O/ab_$1_$2_$i.json" "$1" "$2" >> $O/ab.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d.get("tokens_vs_reference") or {}
r = d["roofline"]
print(sys.argv[2], "VST=" + sys.argv[3], round(d["value"]), d["ms_per_step"], "gemm_us", r.get("gemm_avg_launch_us"), "scan_us", r.get("avg_launch_us"), "tokens", t.get("clips_identical"))
PY
}
for i in 0 1 2; do ab c2 1; ab c2 0; done
i=0; ab c4 1 --seconds 30; ab c4 0 --seconds 30
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --inproc --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
echo done > $O/DONE
