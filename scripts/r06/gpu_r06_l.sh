#!/bin/bash
# r06l: the octet kernel's epilogue without per-block bias loads (the wave's row biases by two scalar
# block loads; a load between two column blocks' stores had waited for all the stores before it) and
# the K-tile-0 offsets read before the first DMA; tests first, then an interleaved A/B against
# lib_eb0 (the round-5 epilogue) and two stagger probes (the first round's second workgroup per CU
# started ~16k / ~32k cycles late).
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_octets.py \
  tests/test_gpu_fp32_guard.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_wpack.py \
  tests/test_gpu_layers.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_eb0" "RRAM_LIB_DIR=$L/lib_st2" "RRAM_LIB_DIR=$L/lib_st4" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
