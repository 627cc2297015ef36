#!/bin/bash
# GPU session: new parallel test, headline bench, each secondary workload, kernel-trace profile.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_gpu_parallel.py tests/test_gpu_layers.py tests/test_gpu_kernels.py} -m gpu -q -x > $O/pytest_par.log 2>&1 || exit $?
timeout -k 10 120 python scripts/kbench.py --only inject && timeout -k 10 120 python scripts/kbench.py --only micro > $O/kbench_inject.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench.json 2> $O/bench.err || exit $?
for w in ${WORKLOADS:-cifar10_quick_mc lenet_train cifar10_full_train googlenet_sweep}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${WSTEPS:-10} --warmup 3 > $O/w_$w.json 2> $O/w_$w.err || exit $?
done
if [ "${PROFILE:-1}" = 1 ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || exit $?
fi
echo done
