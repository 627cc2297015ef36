#!/bin/bash
# k_conv_patch stage-count A/B (2 stages x 2 workgroups/CU vs 3 stages x 1) after the parity tests
set -o pipefail
O=gpurun_out/patch2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for v in 2 3; do RRAM_CONV_PATCH_NST=$v timeout -k 10 200 python scripts/kbench.py --only gemm > $O/kb_$v.txt 2>&1 || exit 1; done
for r in 1 2; do for v in 2 3; do RRAM_CONV_PATCH_NST=$v timeout -k 10 200 python bench.py --no-cpu-baseline --profile-layers > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1; done; done
echo done
