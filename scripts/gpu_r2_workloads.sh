#!/bin/bash
# GPU session: the multi-rank rehearsal tests, then every bench workload once
# (headline + the other BASELINE configs), JSON lines into gpurun_out/r02w/.
set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_par.log 2>&1; rc=$?
tail -3 $O/pytest_par.log; [ $rc -eq 0 ] || exit $rc
for w in alexnet_mc cifar10_quick_mc lenet_mc lenet_train cifar10_full_train googlenet_sweep; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/w_$w.json 2> $O/w_$w.err || { echo "fail $w"; tail -5 $O/w_$w.err; exit 1; }
  cut -c1-220 $O/w_$w.json
done
echo done
