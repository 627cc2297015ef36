#!/bin/bash
# r05ag: the accuracy kernels' batched class loads: the tests that touch
# accuracy, then a kernel trace of the headline bench (k_accuracy_fused was
# 10.0 us per launch in r05u_bench_kernel_stats.csv).
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_host.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --no-cpu-baseline > $R/$O/bench.json 2> $R/$O/bench.err ) || exit 1
python3 - $O/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("accuracy", "softmax")):
        print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
echo done
