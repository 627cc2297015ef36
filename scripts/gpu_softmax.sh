#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/sm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread -k "softmax or mc or MC or alexnet" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.json 2> $O/kt.err || exit 1
grep -h "softmax" $O/kt/run_kernel_stats.csv | cut -c1-140
