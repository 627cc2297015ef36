#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lrn or octet or alexnet" > $O/pytest_r3i.log 2>&1; rc=$?
tail -2 $O/pytest_r3i.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_r3i.log | head; exit $rc; }
REPS=2 ./scripts/ab.sh - || exit 1
for f in gpurun_out/ab/v1_r*.err; do grep -E "pool1|pool2" $f | tr -s ' ' | tr '\n' ' '; echo; done
