#!/bin/bash
# Round-end record on one box: GPU suite, smoke, headline bench line (CPU
# baseline included), rocprofv3 kernel-trace summary and PMC passes of the
# bench command (+ the per-kernel traffic table), the other configs' lines.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=${O:-gpurun_out}; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-300 $O/bench.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || exit $?
timeout -k 10 900 ./scripts/pmc.sh $O/pmc > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 scripts/pmc_traffic.py $O/pmc > $O/pmc_traffic.json && python3 scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt
for w in cifar10_quick_mc cifar10_full_train googlenet_sweep lenet_mc lenet_train; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 > $O/wl_$w.json 2> $O/wl_$w.err || { tail -5 $O/wl_$w.err; exit 1; }
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof_gn_bench.json 2> $R/$O/prof_gn.err ) || exit $?
echo done
