#!/bin/bash
# r06o: the solver's per-iteration clears in one launch (rram_zero_pair: the flat parameter diff and the
# Fail counters); solver / graph / DP / config tests, the C4 kernel sequence, an interleaved C4 line.
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_host.py \
  tests/test_gpu_graph.py tests/test_gpu_native_dp.py tests/test_gpu_solver_kat.py tests/test_gpu_parallel.py \
  tests/test_gpu_configs.py tests/test_gpu_strategy.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4 -o run --output-format csv -- python3 $R/bench.py --workload cifar10_full_train --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c4.json 2> $R/$O/c4.err ) || exit 1
python3 scripts/kernel_sequence.py $O/c4 cifar10_full_train > $O/c4_sequence.txt || exit 1
cat $O/c4_sequence.txt
L=$PWD/rram-caffe-simulation_amd
for r in 1 2 3; do
  for v in - "RRAM_LIB_DIR=$L/lib_fills"; do
    envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
    timeout -k 10 300 env "${envs[@]}" python bench.py --workload cifar10_full_train --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'])" $O/c4.json "$v"
  done
done
