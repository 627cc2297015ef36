#!/bin/bash
# stride-1 data gradient as a flipped-kernel forward convolution (RRAM_DX_FWD):
# parity tests, full GPU suite, C4 / LeNet-train A/B vs the data GEMM + col2im.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "bwd" --timeout 120 --timeout-method thread > $O/tests_bwd.log 2>&1; rc=$?
tail -2 $O/tests_bwd.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_bwd.log | head -40; exit $rc; }
for v in 0 1 0 1; do
  timeout -k 10 300 env RRAM_DX_FWD=$v python bench.py --workload cifar10_full_train --steps 30 --warmup 5 --no-cpu-baseline > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); print('C4 dxfwd=$v', d['value'], d['ms_per_step'])"
done
for v in 0 1; do
  timeout -k 10 300 env RRAM_DX_FWD=$v python bench.py --workload lenet_train --steps 30 --warmup 5 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('LeNet dxfwd=$v', d['value'], d['ms_per_step'])"
done
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --workload cifar10_full_train --steps 50 --warmup 5 --no-cpu-baseline > $R/$O/c4p.json 2> $R/$O/c4p.err) || { tail -5 $O/c4p.err; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp $f $O/c4_kernel_stats.csv; head -25 $O/c4_kernel_stats.csv | cut -c1-150
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1; rc=$?
tail -2 $O/tests_all.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_all.log | head -40; exit $rc; }
