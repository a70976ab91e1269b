#!/bin/bash
# r05e: module victims from tools/diag/stft_surgery.py (stft.hip's SLP build with packed-fp32 forms
# rewritten as scalar pairs, one class at a time) in the interference sequence of r05c: which form,
# removed alone, removes the perturbation?  none (pipeline check), all, opsel, neg, plain.
set -uo pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
for m in none all opsel neg plain; do
  VICTIM_HSACO=tools/_variants/surgery/stft_$m.hsaco timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 > $O/seq_$m.txt 2>&1 || { echo "seq $m rc $?"; tail -8 $O/seq_$m.txt; exit 1; }
  echo "$m: $(grep 'module kernel alone' $O/seq_$m.txt) | $(grep aggressor $O/seq_$m.txt)"
done
