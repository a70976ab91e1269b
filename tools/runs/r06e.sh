#!/bin/bash
# r06e: scan upper-stack register levels A/B (rotated order, warmed chip), then the GPU suite, smoke, the
# default bench line and a 2-rank rehearsal of the N>1 path on this one GPU (gloo, --no-scatter).
set -uo pipefail
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/scan_ab_libs.py 6 32:501,16:501 velocity-asr_amd/velocity_asr/lib/libvasr_hip.so tools/_variants_scan/lib_0_up4.so tools/_variants_scan/lib_1_up3.so tools/_variants_scan/lib_2_nocache.so > $O/ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc $?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('c2', d['value'], d['ms_per_step'], d['config']['schedule'], r['avg_launch_us'], r['frac'], r.get('frac_at_gated_bytes'), d['kernels'], d['cpu_baseline']['value'], d['tokens_vs_reference']['all_ranks_pass'], d['machine']['clock_ghz'])"
VASR_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-scatter > $O/n2.json 2> $O/n2.err || { echo "n2 rc $?"; tail -5 $O/n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2.json')); print('n2', d['value'], d['n_gpus'], d['ms_per_step'], d['tokens_vs_reference']['all_ranks_pass'], d['with_scatter'], d['config']['parallelism'])"
