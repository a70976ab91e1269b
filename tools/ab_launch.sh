set -euo pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --inproc --no-cpu-baseline --roofline-steps 1 > gpurun_out/ab_inproc_$i.json 2>/dev/null
timeout -k 10 300 python bench.py --no-cpu-baseline --roofline-steps 1 > gpurun_out/ab_launch_$i.json 2>/dev/null
done
