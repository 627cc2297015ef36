#!/bin/bash
# r06v2: persistent GoogLeNet conv1 kernel (k_conv_s2p_x6, weights held in registers, double-buffered input
# slots) against the one-tile-per-workgroup k_conv_s2_x6 (lib_s2np: RRAM_S2_PERSIST=0): tests, standalone
# time (interleaved), GoogLeNet trace.
set -o pipefail
O=gpurun_out/r06v2; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$PWD/rram-caffe-simulation_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_x6_range.py tests/test_gpu_fp32_guard.py -k "s2 or bf16x6 or range or guard" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/s2_check.py > $O/s2p_$i.json 2>> $O/s2.err || exit 1
  RRAM_LIB_DIR=$L/lib_s2np timeout -k 10 120 python3 scripts/s2_check.py > $O/s2np_$i.json 2>> $O/s2.err || exit 1
  echo "persistent $(cat $O/s2p_$i.json)  one-per-wg $(cat $O/s2np_$i.json)"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/gn.json 2> $R/$O/gn.err ) || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
grep -E "k_conv_s2" $O/prof_gn/*kernel_stats.csv | cut -c1-160
