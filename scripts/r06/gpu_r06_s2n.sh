#!/bin/bash
# r06s2n: GoogLeNet conv1 k_conv_s2_x6 on 64 x 128 tiles at three workgroups per CU (lib_s2n1, RRAM_S2_NBW=1)
# vs 64 x 256 at two (default): the s2 tests under lib_s2n1, standalone time and GoogLeNet per-layer, interleaved.
set -o pipefail
O=gpurun_out/r06s2n; mkdir -p $O
L=$PWD/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_s2n1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_x6_range.py -k "s2 or engine_bf16x6 or conv7s2" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python3 scripts/s2_check.py > $O/def_$i.json 2>> $O/s2.err || exit 1
  RRAM_LIB_DIR=$L/lib_s2n1 timeout -k 10 120 python3 scripts/s2_check.py > $O/n1_$i.json 2>> $O/s2.err || exit 1
  echo "256: $(cat $O/def_$i.json)  128: $(cat $O/n1_$i.json)"
done
for i in 1 2; do
  timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_def_$i.txt 2>&1 || exit 1
  RRAM_LIB_DIR=$L/lib_s2n1 timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_n1_$i.txt 2>&1 || exit 1
done
for f in $O/gn_def_1.txt $O/gn_n1_1.txt $O/gn_def_2.txt $O/gn_n1_2.txt; do echo "$f: $(grep 'conv1/7x7_s2 ' $f)"; done
