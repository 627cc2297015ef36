#!/bin/bash
# A/B of one env knob: full GPU tests, kbench GEMM table and the headline bench
# line with and without ${AB_ENV} (e.g. AB_ENV=RRAM_CONV_NO_KCU=1).
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_gemm.log 2>&1 || { tail $O/kb_gemm.log; exit 1; }
env ${AB_ENV} timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_gemm_b.log 2>&1 || { tail $O/kb_gemm_b.log; exit 1; }
paste $O/kb_gemm.log $O/kb_gemm_b.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err || { tail $O/bench_a.err; exit 1; }
env ${AB_ENV} timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err || { tail $O/bench_b.err; exit 1; }
cut -c1-330 $O/bench_a.json $O/bench_b.json
