#!/bin/bash
# r05ah: x6 split-K up to 32 splits of >= 4 K-tiles (lib_sp32: fc8 256 x 1000
# x 4096 moves from the fp32 engine's 16 splits to the x6 kernel's 32) vs
# this tree (<= 16 splits of >= 8 K-tiles: fc8 stays on the fp32 engine):
# GEMM / IP / guard tests on lib_sp32, then the interleaved A/B.
set -o pipefail
O=gpurun_out/r05ah; mkdir -p $O
L=$GRAFT_REPO_ROOT/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_sp32 timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
PROFILE_FLAG= REPS=3 scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_sp32" || exit 1
echo done
