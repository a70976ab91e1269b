#!/bin/bash
# r05c: which feature of stft.hip's SLP-packed build perturbs it beside the mel -> conv GEMM sequence
# of another stream.  interference_seq.py (aggressor = recorded calls 1,2,3:
# mel_log_norm, gemm_batched, layer_norm; victim = 20 x 20 STFT launches) with
#   A: stft.hip SLP-vectorised as in round 3 (packed ops read DFT constants from SGPR pairs,
#      8 of them overwritten by s_mov within 2-23 instructions; tools/isa/isa_scan.py)
#   B: the same SLP build with the constants held in VGPRs (109 packed ops, none reading an SGPR)
#   S: the shipped library (no packed fp32 in the STFT kernel)
# then the pk_sgpr_war micro-benchmark (8 variants incl. RAW/WAR distance 1) and the GPU suite.
set -uo pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
for v in A:tools/_variants/stft_slp.so B:tools/_variants/stft_slp_vconst.so; do
  n=${v%%:*}; lib=${v#*:}
  VASR_LIB=$lib timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 > $O/seq_$n.txt 2>&1 || { echo "seq $n rc $?"; tail -5 $O/seq_$n.txt; exit 1; }
  grep aggressor $O/seq_$n.txt
done
timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 > $O/seq_S.txt 2>&1 || { echo "seq S rc $?"; exit 1; }
grep aggressor $O/seq_S.txt
timeout -k 10 300 ./tools/ubench/bin/pk_sgpr_war 20 4000 20000 > $O/pk_sgpr_war.txt 2>&1 || { echo "ubench rc $?"; exit 1; }
cat $O/pk_sgpr_war.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['machine'], d['roofline']['avg_launch_us'], d['config']['schedule'], d['warmup_tokens_vs_reference']['all_ranks_pass'])"
