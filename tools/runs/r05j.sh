#!/bin/bash
# r05j: the C2 step's time course within bursts (tools/diag/step_course.py).
set -uo pipefail
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag/step_course.py > $O/step_course.txt 2>&1 || { echo "rc $?"; tail -5 $O/step_course.txt; exit 1; }
cat $O/step_course.txt
