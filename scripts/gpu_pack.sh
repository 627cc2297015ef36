#!/bin/bash
# octet pack kernel: parity tests + kernel-trace of the bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pack
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
grep -o '"value": [0-9.]*' $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.json 2> $O/kt.err || exit 1
echo ok
