#!/bin/bash
# cb16 paired-block epilogue stores: tests, PMC traffic, bench A/B.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_octets.py tests/test_gpu_wpack.py tests/test_gpu_fp32_guard.py tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
mkdir -p gpurun_out/pmcab
KF="cb" bash scripts/gpu_pmc_ab.sh - 2>&1 | grep -v "declare -x" || exit 1
grep -E "conv_cb" gpurun_out/pmcab/v1.txt | grep -E "grid=   786432|grid=   173056" | sed -E 's/SQ_WAVE.*(FETCH_SIZE=[^ ]+ WRITE_SIZE=[^ ]+).*/\1/'
REPS=3 bash scripts/ab.sh - || exit 1
