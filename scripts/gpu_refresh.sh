#!/bin/bash
# GPU session: LRN/pool parity, per-layer bench, secondary workloads, PMC passes.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_layers.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_layers.json 2> $O/bench_layers.err || exit $?
for w in ${WORKLOADS:-lenet_mc cifar10_quick_mc lenet_train cifar10_full_train googlenet_sweep}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${WSTEPS:-10} --warmup 3 > $O/w_$w.json 2> $O/w_$w.err || exit $?
done
if [ "${PMC:-1}" = 1 ]; then
  bash scripts/pmc.sh gpurun_out/pmc || exit $?
fi
echo done
