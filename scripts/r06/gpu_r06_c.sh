#!/bin/bash
# r06c: where the 3x3 octet kernel's cycles go (s_memtime stamp build
# lib_cbstamp, scripts/cb_stamp.py) for conv3 / conv4 / conv5.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_cbstamp timeout -k 10 300 python scripts/cb_stamp.py > $O/cb_stamp.txt 2>&1; rc=$?
cat $O/cb_stamp.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/graph_release_probe.py > $O/graph_probe.txt 2>&1; rc=$?
cat $O/graph_probe.txt; exit $rc
