#!/bin/bash
# r06z: the 1x1 kernels' convolution-output fold (GoogLeNet reductions write only their octet companion):
# octets-only / fold / C5 / conv tests, then the GoogLeNet sweep's trace and per-layer times.
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layers.py \
  tests/test_gpu_configs.py tests/test_gpu_conv1x1.py tests/test_gpu_octets.py tests/test_gpu_graph.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/gn.json 2> $R/$O/gn.err ) || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_layers.txt 2>&1 || exit 1
head -2 $O/gn_layers.txt; grep reduce $O/gn_layers.txt | head -12
