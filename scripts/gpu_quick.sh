#!/bin/bash
# Quick GPU iteration: GPU tests, conv/IP GEMM micro-bench (with and without
# the gather table), headline bench line.  Each step has its own time limit.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_gemm.log 2>&1 || { tail $O/kb_gemm.log; exit 1; }
RRAM_CONV_NO_TABLE=1 timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_gemm_notable.log 2>&1 || exit 1
paste $O/kb_gemm.log $O/kb_gemm_notable.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_quick.json 2> $O/bench_quick.err || { tail $O/bench_quick.err; exit 1; }
cat $O/bench_quick.json
