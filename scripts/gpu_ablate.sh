#!/bin/bash
# Diagnostic ablation A/B (wrong-result builds, timing only): kbench GEMM shapes
# for the base library and each lib_<V> variant, interleaved twice.
set -o pipefail
O=gpurun_out/ablate
mkdir -p $O
for rep in 1 2; do
for v in base ${VARIANTS}; do
  d=rram-caffe-simulation_amd/lib_$v; [ $v = base ] && d=rram-caffe-simulation_amd/lib
  RRAM_LIB_DIR=$PWD/$d timeout -k 10 120 python scripts/kbench.py --only gemm > $O/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -5 $O/kb_${v}_$rep.log; exit 1; }
  echo "$v.$rep $(grep -E '_ms' $O/kb_${v}_$rep.log | awk '{printf "%s=%s ", $1, $2}')"
done
done
