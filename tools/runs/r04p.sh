#!/bin/bash
# r04p: HEAD-configuration profile evidence: rocprofv3 kernel trace + stats and
# HBM counter passes of the default bench command, SQ counters of the bench's scan launch (16 clips, one utterance group),
# MFMA counters of the GEMM shapes at M = 8016 (one utterance group).
set -uo pipefail
export TMPDIR=/tmp
step() {  # step NAME CMD...: stop at the first failing GPU step
  local n=$1; shift
  "$@"; local rc=$?
  echo "$n rc $rc"
  [ $rc -eq 0 ] || exit $rc
}
step profile bash tools/profile.sh r04p --steps 10 --warmup 3 --no-cpu-baseline
step scan_pmc bash tools/pmc_kernel.sh r04p_scan16 python3 tools/scan_bench.py 16 501 384 64 2 20
step mfma bash tools/pmc_mfma.sh r04p 8016
ls gpurun_out/prof_r04p gpurun_out/pmc_r04p_scan16 gpurun_out/mfma_r04p_8016
