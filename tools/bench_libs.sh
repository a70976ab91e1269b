#!/bin/bash
# End-to-end bench of the default library and each variant in tools/_variants/ (VASR_LIB), interleaved twice.
set -euo pipefail
mkdir -p gpurun_out
run() {
  local name=$1 lib=$2
  if [ -n "$lib" ]; then VASR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bl_$name.log 2>&1
  else timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bl_$name.log 2>&1; fi
  tail -n 1 gpurun_out/bl_$name.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print('$name', d['value'], d['ms_per_step'], k['scan']['avg_launch_us'], k['gemm']['avg_launch_us'])"
}
for rep in 1 2; do
  run base ""
  for lib in tools/_variants/*.so; do run "$(basename $lib .so)" "$PWD/$lib"; done
done
