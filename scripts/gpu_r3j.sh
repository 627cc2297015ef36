#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_host.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "accuracy or mc or c3 or c1" > $O/pytest_r3j.log 2>&1; rc=$?
tail -2 $O/pytest_r3j.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_r3j.log | head; exit $rc; }
REPS=2 ./scripts/ab.sh - || exit 1
