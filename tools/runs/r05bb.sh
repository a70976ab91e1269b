#!/bin/bash
# N > 1 rehearsal at the final HEAD: two ranks pinned to the one GPU (bench.py's torchrun path, gloo
# timing group, no scatter leg since RCCL refuses two ranks on one device), and the distributed GPU tests.
set -uo pipefail
O=gpurun_out/r05bb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 240 --timeout-method thread > $O/dist_tests.txt 2>&1; rc=$?
tail -2 $O/dist_tests.txt; [ $rc -eq 0 ] || exit $rc
VASR_BENCH_DEVICE=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-scatter --roofline-steps 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc $?"; tail -20 $O/n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/n2.json')); print('n2', d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('schedule', {}).get('chosen_streams'), d['tokens_vs_reference']['all_ranks_pass'])"
