#!/bin/bash
# r04l: which ops of group 0's pipeline prefix perturb group 1's STFT (index selections), and does
# the perturbation follow the tile GEMM's staging form (asm LDS-DMA / compiler LDS-DMA builtin /
# register staging; tools/_variants built by tools/build_variant_lib.sh -DVASR_X3_STAGE=1|2)?
set -uo pipefail
O=gpurun_out/r04l
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -5 $O/$n.txt; exit $rc; }
}
run seq_head timeout -k 10 300 python -u tools/diag/interference_seq.py 10 10 4 3 2,3 0,1,3 2, 0,1,2 1,2,3 12
VASR_LIB=tools/_variants/x3builtin.so run seq_builtin timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 4 2,3 12
VASR_LIB=tools/_variants/x3reg.so run seq_reg timeout -k 10 200 python -u tools/diag/interference_seq.py 10 10 4 2,3 12
grep -h aggressor $O/*.txt
