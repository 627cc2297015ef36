#!/bin/bash
# round-3 workload lines (C2 / C4 / C5 with roofline + cpu_baseline) and the C5 tests
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c5" > $O/pytest_c5.log 2>&1; rc=$?
tail -3 $O/pytest_c5.log; [ $rc -eq 0 ] || exit $rc
for w in cifar10_quick_mc cifar10_full_train googlenet_sweep lenet_mc lenet_train; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 > $O/wl_$w.json 2> $O/wl_$w.err || { tail -5 $O/wl_$w.err; exit 1; }
  cut -c1-400 $O/wl_$w.json
done
