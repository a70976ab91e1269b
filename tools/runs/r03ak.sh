#!/bin/bash
# r03ak: launch floor of graph kernel nodes and one-utterance latency under HIP runtime knobs.
set -uo pipefail
O=gpurun_out/r03ak
mkdir -p $O
run() {  # tag, env assignments...
  tag=$1; shift
  env "$@" timeout -k 10 60 python tools/diag/launch_floor.py > $O/floor_$tag.txt 2>&1 || return 1
  env "$@" timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 50 --warmup 10 --no-cpu-baseline --roofline-steps 2 > $O/b1_$tag.json 2> $O/b1_$tag.err || return 1
  python3 -c "import json; d=json.loads(open('$O/b1_$tag.json').read().strip().splitlines()[-1]); print('$tag', open('$O/floor_$tag.txt').read().strip().splitlines()[-1], 'b1 ms', d['ms_per_step'])" >> $O/knobs.txt
}
run base X=1 && run devkarg1 HIP_FORCE_DEV_KERNARG=1 && run devkarg0 HIP_FORCE_DEV_KERNARG=0 && run batch1 DEBUG_HIP_GRAPH_BATCH_SIZE=1 && run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run fgs ROC_USE_FGS_KERNARG=1 && run sysscope0 ROC_SYSTEM_SCOPE_SIGNAL=0 && run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run base2 X=2
cat $O/knobs.txt
