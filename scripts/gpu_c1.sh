#!/bin/bash
# conv1 iteration: accuracy + time of the conv1 kernel, the conv tests, the bench line
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 180 python scripts/conv1_check.py > $O/c1.json 2>&1; rc=$?; cat $O/c1.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or alexnet or c3 or octet" > $O/pytest_c1.log 2>&1; rc=$?
tail -3 $O/pytest_c1.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest_c1.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_c1.json'));print(d['value'], d['roofline']['layers']['conv1'])"
