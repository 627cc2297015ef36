#!/bin/bash
# r06ra: row-aligned per-image tiles for the two-per-CU octet kernel (CbPlan.tp, ConvGeom.tpitch):
# correctness under lib_rowalign (RRAM_CB_ROWALIGN=2: the row-aligned plan wherever it fits), then GoogLeNet
# per-layer times interleaved default / forced, then the AlexNet bench line for both.
set -o pipefail
O=gpurun_out/r06ra; mkdir -p $O
L=$PWD/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_rowalign timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_octets.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_fp32_guard.py \
  -k "conv or octet or c5 or guard or patch" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_def_$i.txt 2>&1 || exit 1
  RRAM_LIB_DIR=$L/lib_rowalign timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_ra_$i.txt 2>&1 || exit 1
done
for f in $O/gn_def_1.txt $O/gn_ra_1.txt $O/gn_def_2.txt $O/gn_ra_2.txt; do
  echo "$f: $(sed -n 2p $f)"; grep -E "conv2/3x3 |inception_3a/3x3 |inception_3b/3x3 |inception_4./3x3 |5x5 " $f | head -14
done
REPS=2 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_rowalign" > $O/ab.txt 2>&1; cat $O/ab.txt
