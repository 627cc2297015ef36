#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
for d in 0 2 4; do
  RRAM_C1_DIAG=$d timeout -k 10 120 python scripts/conv1_check.py > $O/c1d_$d.json 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
  echo "diag $d: $(tail -1 $O/c1d_$d.json)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_wpack.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wpack or cached or pack or conv_fault or c3" > $O/pytest_r3c.log 2>&1; rc=$?
tail -15 $O/pytest_r3c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_r3c.json 2> $O/bench_r3c.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_r3c.json'));print(d['value'], d['roofline']['frac'], d['roofline']['layers'])"
