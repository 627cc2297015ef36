#!/bin/bash
# r06b: the native RCCL data-parallel path (C driver + Python view, world 1),
# the bench's RCCL world-1 runs through it, the graph tests (ADVICE r05
# release-caches case); then the round-6 starting point: headline bench line
# with per-layer times and a kernel-trace summary.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_native_dp.py tests/test_gpu_parallel.py \
  "tests/test_gpu_solver_kat.py::test_least_squares_update_rccl_world1" tests/test_gpu_graph.py > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --profile-layers > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || exit $?
echo done
