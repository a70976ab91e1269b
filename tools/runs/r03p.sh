#!/bin/bash
# r03p: MFMA counters of the HEAD step's GEMMs / tails after the rows engine + 12-wave tail (row N1)
set -euo pipefail
bash tools/pmc_mfma.sh r03p 8016
