#!/bin/bash
# r06pb: banded 3 x 3 max pool for planes over 4096 elements (k_pool_band3; GoogLeNet pool1): pooling / layer /
# C5 tests, then GoogLeNet per-layer times.
set -o pipefail
O=gpurun_out/r06pb; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layers.py \
  tests/test_gpu_pooling_kat.py tests/test_gpu_configs.py -k "pool or c5 or googlenet" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/gn_layers.py --maps 6 --top 200 > $O/gn_layers.txt 2>&1 || exit 1
sed -n 2p $O/gn_layers.txt; grep -E "pool1/|pool3/|pool4/" $O/gn_layers.txt
