#!/bin/bash
# cb16 cross-pair + Concat fold check: tests under RRAM_CB16=3, the headline
# A/B of the cb16 variants, GoogLeNet sweep lines with and without the fold.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
[ -n "$SKIP_AB" ] || timeout -k 10 900 env RRAM_CB16=3 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py tests/test_gpu_wpack.py tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "err / sum" $O/tests.log; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
[ -n "$SKIP_AB" ] || { REPS=2 scripts/ab.sh "RRAM_CB16=0" "RRAM_CB16=1" "RRAM_CB16=3" || exit 1; }
i=0
for v in "RRAM_FUSE_CONCAT=0 RRAM_CB16=1" "RRAM_CB16=1" "RRAM_FUSE_CONCAT=0 RRAM_CB16=1" "RRAM_CB16=1" "RRAM_CB16=3"; do
  i=$((i + 1)); read -ra envs <<< "$v"
  timeout -k 10 300 env "${envs[@]}" python bench.py --workload googlenet_sweep --steps 3 --warmup 1 --no-cpu-baseline > $O/gn_$i.json 2> $O/gn_$i.err || { tail -5 $O/gn_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/gn_$i.json')); print('googlenet [$v]', d['value'], d['ms_per_step'])"
done
