#!/bin/bash
# LRN + max-pool LDS pitch: tests, bench layer table, PMC of the band kernel.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_configs.py tests/test_gpu_fp32_guard.py -m gpu -x -q -k "lrn or pool or alexnet or c5 or fp32" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
REPS=2 bash scripts/ab.sh - || exit 1
grep -E "pool1|pool2" gpurun_out/ab/v1_r2.err
R=$GRAFT_REPO_ROOT
KFILTER=lrn bash scripts/pmc_kernel.sh $O/pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
grep -E "lrn_maxpool" $O/pmc.txt | cut -c1-700
python3 scripts/pmc_clock.py $O/pmc.txt | grep -E "lrn"
