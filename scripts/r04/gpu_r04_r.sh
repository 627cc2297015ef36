#!/bin/bash
# C4 (CIFAR-10 full training) kernel trace: launches per iteration and busy time.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --workload cifar10_full_train --steps 50 --warmup 5 --no-cpu-baseline > $R/$O/c4.json 2> $R/$O/c4.err) || { tail -5 $O/c4.err; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp $f $O/c4_kernel_stats.csv; head -30 $O/c4_kernel_stats.csv | cut -c1-170
f2=$(find $O/kt -name "*kernel_trace.csv" | head -1); python3 - "$f2" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0, t1 = int(rows[len(rows)//3]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
mid = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in mid)
print("kernels", len(mid), "span us", (t1 - t0) / 1e3, "busy us", busy / 1e3, "busy frac", busy / (t1 - t0))
PY
