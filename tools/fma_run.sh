set -o pipefail
mkdir -p gpurun_out/fma
timeout -k 10 400 python -u -m pytest tests/test_scan_fma.py tests/test_gpu_parity.py -k "scan or fma" -x -q --timeout 120 --timeout-method thread > gpurun_out/fma/pytest.log 2>&1 || exit 1
for m in 0 2; do timeout -k 10 60 python tools/scan_bench.py 16 501 384 64 $m 100 >> gpurun_out/fma/scan.txt 2>&1 || exit 1; timeout -k 10 60 python tools/scan_bench.py 32 501 384 64 $m 100 >> gpurun_out/fma/scan.txt 2>&1 || exit 1; done
for r in 1 2; do for f in 0 1; do VASR_SCAN_FMA=$f timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fma/bench_fma$f.$r.json 2>/dev/null || exit 1; done; done
