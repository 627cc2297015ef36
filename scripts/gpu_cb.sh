#!/bin/bash
# A/B of the channel-octet bf16x6 convolution (k_conv_cb_x6): conv parity
# tests, then the bench's per-layer times with it off (RRAM_CONV_CB=0) and on.
set -o pipefail
O=gpurun_out/cb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rP --timeout 300 --timeout-method thread -k "patch or engine or conv" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit $rc; }
grep "bf16x6 .*e-" $O/pytest.log | head -8
for x in 0 1; do
  RRAM_CONV_CB=$x timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_$x.json 2> $O/layers_$x.txt || exit 1
  cut -c1-200 $O/bench_$x.json; grep -E "conv[1-5] " $O/layers_$x.txt
done
