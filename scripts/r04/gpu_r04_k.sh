#!/bin/bash
# 256-byte octet planes (cb16 conflicts) + 1x1 per-shape variant: tests, bench A/B, PMC of the cb kernels.
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wpack.py tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py tests/test_gpu_conv1x1.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
REPS=3 bash scripts/ab.sh - || exit 1
R=$GRAFT_REPO_ROOT
bash scripts/pmc_kernel.sh $O/pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
grep -E "conv_cb" $O/pmc.txt | cut -c1-900
for v in 1 1; do
  timeout -k 10 300 python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5.json')); print('C5', d['value'], d['ms_per_step'], d['roofline'].get('achieved'))"
done
