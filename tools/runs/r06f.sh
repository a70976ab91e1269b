#!/bin/bash
# r06f: the round-6 evidence at HEAD: rocprofv3 kernel trace + FETCH/WRITE passes of the default bench
# (tools/profile.sh), MFMA counters of the GEMM / tail kernels at the bench's M (tools/pmc_mfma.sh), SQ
# counters of the 32-clip scan launch, ungated (the bench's) and gated.
set -uo pipefail
export TMPDIR=/tmp
bash tools/profile.sh r06f || { echo "profile rc $?"; exit 1; }
echo profile done
bash tools/pmc_mfma.sh r06f 16032 || { echo "pmc_mfma rc $?"; exit 1; }
echo mfma done
SCAN_UNGATED=1 bash tools/pmc_kernel.sh r06f_scan32u python3 tools/scan_bench.py 32 501 384 64 2 20 || { echo "pmc scan rc $?"; exit 1; }
bash tools/pmc_kernel.sh r06f_scan32g python3 tools/scan_bench.py 32 501 384 64 2 20 || { echo "pmc scan g rc $?"; exit 1; }
SCAN_UNGATED=1 bash tools/pmc_kernel.sh r06f_scan32x30 python3 tools/scan_bench.py 32 1501 384 64 2 10 || { echo "pmc scan c4 rc $?"; exit 1; }
echo pmc done
mkdir -p gpurun_out/r06f
VASR_PARITY_LOG=gpurun_out/r06f/parity_headline.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "headline or full_batch" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06f/headline_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r06f/headline_tests.txt; cat gpurun_out/r06f/parity_headline.jsonl; [ $rc -eq 0 ] || exit $rc
