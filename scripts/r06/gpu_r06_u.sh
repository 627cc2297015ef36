#!/bin/bash
# r06u2: the separable TEST-phase 3 x 3 max pool (k_pool_planes_sep3): layer / pooling / C5 / graph tests,
# then the GoogLeNet sweep's kernel trace.
set -o pipefail
O=gpurun_out/r06u2; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layers.py \
  tests/test_gpu_pooling_kat.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_octets.py \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/gn.json 2> $R/$O/gn.err ) || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
grep -E "k_pool_planes" $O/prof_gn/*kernel_stats.csv | cut -c1-160
