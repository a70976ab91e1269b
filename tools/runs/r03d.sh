#!/bin/bash
# r03d: stream structure x scan decomposition, interleaved, 2 rounds.
set -euo pipefail
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 1100 python tools/ab_matrix.py $O/ab 2 \
  'base||' \
  'one_graph||--streams 1' \
  'one_graph_t32|VASR_SCAN_T=32|--streams 1' \
  'npl2|VASR_SCAN_NPL=2|' \
  'npl2_t32|VASR_SCAN_NPL=2 VASR_SCAN_T=32|' \
  'npl2_t16|VASR_SCAN_NPL=2 VASR_SCAN_T=16|' > $O/ab.out 2>&1
echo done > $O/DONE
