#!/bin/bash
# k_conv_patch bring-up: conv parity tests, then kbench and the headline bench
# with the patch convolution on (default) and off (RRAM_CONV_PATCH=0).
set -o pipefail
O=gpurun_out/patch
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in 1 0; do RRAM_CONV_PATCH=$v timeout -k 10 200 python scripts/kbench.py --only gemm > $O/kb_$v.txt 2>&1 || exit 1; done
for r in 1 2; do for v in 1 0; do RRAM_CONV_PATCH=$v timeout -k 10 200 python bench.py --no-cpu-baseline --profile-layers > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1; done; done
echo done
