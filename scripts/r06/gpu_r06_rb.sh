#!/bin/bash
# r06rb: GoogLeNet conv2's row-aligned plan on 128 x 128 tiles (default) vs 64 x 128 (lib_ra64, RRAM_CB_RA_WR=2):
# conv tests under lib_ra64, then per-layer times interleaved.
set -o pipefail
O=gpurun_out/r06rb; mkdir -p $O
L=$PWD/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_ra64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -k "engine_bf16x6 or patch_shapes" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_def_$i.txt 2>&1 || exit 1
  RRAM_LIB_DIR=$L/lib_ra64 timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_64_$i.txt 2>&1 || exit 1
done
for f in $O/gn_def_1.txt $O/gn_64_1.txt $O/gn_def_2.txt $O/gn_64_2.txt; do
  echo "$f: $(sed -n 2p $f) $(grep 'conv2/3x3 ' $f)"
done
