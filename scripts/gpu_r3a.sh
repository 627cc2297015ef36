#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 180 python scripts/conv1_check.py > $O/c1_ring.json 2>&1; echo "ring rc=$?" >> $O/c1_ring.json
RRAM_WIDE_V1=1 timeout -k 10 180 python scripts/conv1_check.py > $O/c1_v1.json 2>&1 || exit $?
cat $O/c1_ring.json $O/c1_v1.json
grep -q "ring rc=0" $O/c1_ring.json || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
