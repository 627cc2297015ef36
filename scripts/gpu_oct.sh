#!/bin/bash
# Octet-companion session: the octet / conv / C3 parity tests, the bench
# line, and a rocprofv3 kernel-trace summary of the bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/oct
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "octet or patch or engine or conv or c3 or ip or gemm or c2 or c5" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench.json 2> $O/layers.txt || { tail -20 $O/layers.txt; exit 1; }
cut -c1-220 $O/bench.json; grep -E "conv[1-5] |pool[12] " $O/layers.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.json 2> $O/kt.err || exit 1
echo ok
