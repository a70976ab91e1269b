#!/bin/bash
# r04af: gloo timing group -- N = 1 default line x2, the distributed GPU tests (launcher at N = 1
# with the RCCL serving leg), and a 2-rank rehearsal on this one GPU (both ranks on device 0,
# --no-scatter: the gloo barriers / max / token checks of the N > 1 path).
set -uo pipefail
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread > $O/dist.txt 2>&1 || { echo "dist tests failed"; tail -20 $O/dist.txt; exit 1; }
tail -1 $O/dist.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { echo "b$i rc $?"; tail -5 $O/b$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b$i.json')); w=d.get('with_scatter') or {}; print('b$i', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'], w.get('value'), w.get('rank0_tokens_match'), d['config']['parallelism'][:60])"
done
VASR_BENCH_DEVICE=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-scatter --roofline-steps 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc $?"; tail -20 $O/n2.err; exit 1; }
python -c "import json; d=json.load(open('$O/n2.json')); print('n2', d['n_gpus'], d['value'], d['ms_per_step'], d['tokens_vs_reference'], d['graph_tokens_match_eager'])"
