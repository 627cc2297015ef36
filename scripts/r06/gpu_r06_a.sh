#!/bin/bash
# r06a: round-6 starting point on one box: the headline bench line with
# per-layer times, and a kernel-trace summary of the same command.
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --profile-layers > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || exit $?
echo done
