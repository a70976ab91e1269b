set -euo pipefail
mkdir -p gpurun_out
export VASR_PARITY_LOG=$PWD/gpurun_out/parity_margins.jsonl
rm -f $VASR_PARITY_LOG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_scan_fma.py tests/test_ragged.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_margins.log 2>&1
unset VASR_PARITY_LOG
bash tools/profile.sh r02d
