set -euo pipefail
mkdir -p gpurun_out/tailpd
timeout -k 10 120 python tools/tail_bench.py 8016 > gpurun_out/tailpd/pd3.txt 2>&1
for pd in 2 4 5; do VASR_LIB=$PWD/tools/_variants/tailpd$pd.so timeout -k 10 120 python tools/tail_bench.py 8016 > gpurun_out/tailpd/pd$pd.txt 2>&1; done
timeout -k 10 120 python tools/tail_bench.py 8016 > gpurun_out/tailpd/pd3b.txt 2>&1
