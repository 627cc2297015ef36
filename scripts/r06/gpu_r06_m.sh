#!/bin/bash
# r06m: the flipped convolution kernels written by the fused update (rram_update_seg.w_flip) and read
# by the next backward of the same Step call; solver / graph / DP tests first, then the C4 iteration's
# kernel sequence and an interleaved C4 line with the cache on and off (net option conv_flip_cache).
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_host.py \
  tests/test_gpu_graph.py tests/test_gpu_native_dp.py tests/test_gpu_solver_kat.py tests/test_gpu_parallel.py \
  tests/test_gpu_configs.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4 -o run --output-format csv -- python3 $R/bench.py --workload cifar10_full_train --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c4.json 2> $R/$O/c4.err ) || exit 1
python3 scripts/kernel_sequence.py $O/c4 cifar10_full_train > $O/c4_sequence.txt || exit 1
cat $O/c4_sequence.txt
for r in 1 2 3; do
  for v in 1 0; do
    F=""; [ $v = 0 ] && F=--no-conv-flip-cache
    timeout -k 10 300 python bench.py --workload cifar10_full_train --no-cpu-baseline $F > $O/c4_v${v}_r$r.json 2> $O/c4_v${v}_r$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cache', sys.argv[2], d['value'], d['unit'], d['ms_per_step'])" $O/c4_v${v}_r$r.json $v
  done
done
