#!/bin/bash
# rocprofv3 kernel-trace summary of the headline bench command (no PMC).
set -o pipefail
O=gpurun_out
mkdir -p $O
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
for r in rows[:16]:
    n = r["Name"].replace("rram::(anonymous namespace)::", "")[:70]
    print(f"{n:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us {float(r['Percentage']):6.2f}%")
PY
cat $O/prof_bench.json | cut -c1-200
