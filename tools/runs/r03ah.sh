#!/bin/bash
# r03ah: graph replay of utterance group 0 on the caller's stream (no cross-stream events for it) vs every group
# on its own stream: one-utterance latency and C2 A/B.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
for r in 0 1; do
  for k in 0 1; do
    VASR_MAIN_GROUPS=$k timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 100 --warmup 10 --no-cpu-baseline --roofline-steps 1 > $O/b1_k${k}_r$r.json 2> $O/b1_k${k}_r$r.err
  done
done
timeout -k 10 900 python tools/ab_matrix.py $O/ab 3 'k0|VASR_MAIN_GROUPS=0|' 'k1|VASR_MAIN_GROUPS=1|' > $O/ab.txt 2>&1
echo done > $O/DONE
# (VASR_MAIN_GROUPS was a temporary A/B switch in GraphedTranscriber.step; group 0 on the caller's stream is now the code)
