#!/bin/bash
# r05f: the op_sel class of r05e split (v_pk_mov_b32 / dword swaps / high-dword broadcasts), and the
# shipped ln_dwconv kernel (9 v_pk_mov_b32 with op_sel) as the victim of the same aggressors.
set -uo pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
for m in opsel_mov opsel_swap opsel_bcast; do
  VICTIM_HSACO=tools/_variants/surgery/stft_$m.hsaco timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 > $O/seq_$m.txt 2>&1 || { echo "seq $m rc $?"; tail -8 $O/seq_$m.txt; exit 1; }
  echo "$m: $(grep aggressor $O/seq_$m.txt)"
done
VICTIM=4 timeout -k 10 300 python -u tools/diag/interference_seq.py 20 20 1,2,3 2, 3 > $O/seq_lndw.txt 2>&1 || { echo "seq lndw rc $?"; tail -8 $O/seq_lndw.txt; exit 1; }
grep "victim\|aggressor" $O/seq_lndw.txt
