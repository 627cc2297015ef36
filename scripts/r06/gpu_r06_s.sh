#!/bin/bash
# r06s: GoogLeNet conv1 (7 x 7 / 2, 3 channels) on the bf16x6 engine (k_conv_s2_x6); its shape / accuracy /
# range tests, the conv and C5 tests, then the GoogLeNet sweep's kernel trace.
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_x6_range.py tests/test_gpu_fp32_guard.py tests/test_gpu_configs.py tests/test_gpu_layers.py \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/gn.json 2> $R/$O/gn.err ) || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
grep -E "k_conv_s2|k_gemm<1, 4, 2, 1, 0, 7" $O/prof_gn/*kernel_stats.csv | cut -c1-160
