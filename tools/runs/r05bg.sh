#!/bin/bash
# Log-mel CSR entries read 8 at a time before their fmas: output digests on both libraries,
# GPU suite, front-end timings, interleaved one-utterance and C2 lines vs the previous library.
set -uo pipefail
OUT=gpurun_out/r05bg; mkdir -p $OUT
MAIN=velocity-asr_amd/velocity_asr/lib/libvasr_hip.so
OLD=tools/_variants/melold.so
DIG='import sys; sys.path.insert(0, "velocity-asr_amd"); import torch; from velocity_asr import audio as A
g = torch.Generator().manual_seed(3)
for B, S in ((1, 160000), (4, 48000), (3, 16001)):
    x = (torch.randn(B, S, generator=g) * 0.1).cuda()
    m = A.compute_mel_spectrogram(x)
    print(B, S, int(m.contiguous().view(torch.int32).to(torch.int64).sum().item()))'
for lib in $MAIN $OLD; do VASR_LIB=$lib timeout -k 10 120 python -c "$DIG" 2>/dev/null | sed "s/^/$(basename $lib .so) /" >> $OUT/digests.txt; done
cat $OUT/digests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for lib in $MAIN $OLD; do for B in 1 32; do VASR_LIB=$lib timeout -k 10 90 python tools/frontend_bench.py $B 2>/dev/null | sed "s/^/$(basename $lib .so) /" >> $OUT/frontend.txt; done; done
for r in 1 2 3; do
  for lib in $MAIN $OLD; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --inproc --batch 1 --seconds 10 --steps 200 --warmup 20 \
      --no-cpu-baseline --roofline-steps 2 > $OUT/b1.$n.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/b1.$n.$r.json'));print('b1 $n r$r', d['ms_per_step'])" >> $OUT/summary.txt
  done
done
for r in 1 2; do
  for lib in $MAIN $OLD; do
    n=$(basename $lib .so)
    VASR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$n.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/c2.$n.$r.json'));print('c2 $n r$r', d['value'], d['ms_per_step'], d['tokens_vs_reference']['all_ranks_pass'])" >> $OUT/summary.txt
  done
done
cat $OUT/frontend.txt $OUT/summary.txt
