#!/bin/bash
# Interleaved A/B of bench.py under an environment toggle: bash tools/ab_env.sh <tag> VAR "valA valB" [pairs] [bench args]
set -euo pipefail
TAG=$1; VAR=$2; VALS=$3; PAIRS=${4:-2}; shift 4 || true
mkdir -p gpurun_out/ab_$TAG
for r in $(seq 1 $PAIRS); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --inproc --no-cpu-baseline --roofline-steps 2 "$@" \
      > gpurun_out/ab_$TAG/$VAR-$v.$r.json 2> gpurun_out/ab_$TAG/$VAR-$v.$r.err
  done
done
