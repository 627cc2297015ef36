#!/bin/bash
# r06h: where k_conv_cb16_x6's cycles go, conv2 (5x5) and conv3 / conv4 / conv5 (3x3), after the
# round-6 changes (s_memtime stamp build lib_cbstamp, scripts/cb_stamp.py).
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_cbstamp timeout -k 10 300 python scripts/cb_stamp.py > $O/cb_stamp.txt 2>&1; rc=$?
cat $O/cb_stamp.txt; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || exit $?
echo done
