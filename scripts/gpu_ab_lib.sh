#!/bin/bash
# A/B of a compile-time variant library (lib_${V}) against lib/: GPU tests on
# the default build, kbench GEMM table and the bench workloads with both.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
V=${V:?set V}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lib in lib lib_$V; do
  export RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/$lib
  timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_$lib.log 2>&1 || { tail $O/kb_$lib.log; exit 1; }
  echo "$lib $(grep -E '_ms' $O/kb_$lib.log | awk '{printf "%s=%s ", $1, $2}')"
  for w in ${WORKLOADS:-alexnet_mc}; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > $O/b_${lib}_$w.json 2> $O/b_${lib}_$w.err || { tail $O/b_${lib}_$w.err; exit 1; }
    echo "$lib $w $(cut -c1-160 $O/b_${lib}_$w.json)"
  done
done
