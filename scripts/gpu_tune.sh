#!/bin/bash
# Tuning session: parity tests, injection grid sweep, bench with/without
# all-layer events, then PMC passes.  Every GPU step has its own time limit.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_host.py} -m gpu -q -x > $O/pytest_tune.log 2>&1 || exit $?
for g in 2048 8192 1073741824; do
  RRAM_INJECT_GRID=$g timeout -k 10 120 python scripts/kbench.py --only inject > $O/kb_inject_$g.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_t2.json 2> $O/bench_t2.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_t1.json 2> $O/bench_t1.err || exit $?
timeout -k 10 120 python scripts/kbench.py --only gemm > $O/kb_gemm.log 2>&1 || exit $?
if [ "${PMC:-1}" = 1 ]; then
  bash scripts/pmc.sh $O/pmc3 || exit $?
fi
echo done
