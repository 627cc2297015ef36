#!/bin/bash
# A/B the GEMM schedule variants built by `make LIBDIR=lib_<V> OBJDIR=build_<V> VARIANT=-DRRAM_V_<V>`.
set -o pipefail
O=gpurun_out/variants
mkdir -p $O
for v in base ${VARIANTS:-NOSCHED SPREAD PRIO}; do
  d=rram-caffe-simulation_amd/lib_$v; [ $v = base ] && d=rram-caffe-simulation_amd/lib
  RRAM_LIB_DIR=$PWD/$d timeout -k 10 120 python scripts/kbench.py --only gemm > $O/kb_$v.log 2>&1 || { echo "fail $v"; tail -5 $O/kb_$v.log; exit 1; }
  echo "$v $(grep -E '_ms' $O/kb_$v.log | awk '{printf "%s=%s ", $1, $2}')"
done
