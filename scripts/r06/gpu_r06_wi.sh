#!/bin/bash
# r06wi: whole-image octet tiles for planes of < 64 positions (GoogLeNet's 7 x 7 stage onto the bf16x6 octet
# kernel): conv / octet / fold / C5 / guard tests, GoogLeNet per-layer times and trace, AlexNet bench line.
set -o pipefail
O=gpurun_out/r06wi; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_octets.py tests/test_gpu_layers.py tests/test_gpu_configs.py tests/test_gpu_fp32_guard.py \
  tests/test_gpu_x6_range.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_layers.txt 2>&1 || exit 1
sed -n 2p $O/gn_layers.txt; grep -E "inception_5./(3x3|5x5) " $O/gn_layers.txt
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/gn.json 2> $R/$O/gn.err ) || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['engines'])"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
