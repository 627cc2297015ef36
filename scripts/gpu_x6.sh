#!/bin/bash
# A/B of the bf16x6 patch convolution: parity tests on the conv kernels, then
# the bench with per-layer times with the x6 path off and on.
set -o pipefail
O=gpurun_out/x6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv or c3_" > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do
  RRAM_CONV_X6=$x timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_$x.json 2> $O/layers_$x.txt || exit 1
  cut -c1-200 $O/bench_$x.json
done
