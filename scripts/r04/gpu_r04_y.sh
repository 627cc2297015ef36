#!/bin/bash
# C4 backward: 16-byte im2col, one-pass chunks (256 images), parallel bias reductions.
set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "bwd or im2col or bias" --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for w in cifar10_full_train lenet_train cifar10_full_train lenet_train; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --workload cifar10_full_train --steps 50 --warmup 5 --no-cpu-baseline > $R/$O/c4p.json 2> $R/$O/c4p.err) || { tail -5 $O/c4p.err; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp $f $O/c4_kernel_stats.csv
python3 - <<'PY'
import csv, re
for r in list(csv.DictReader(open("gpurun_out/r04y/c4_kernel_stats.csv")))[:16]:
    nm = re.sub(r"rram::\(anonymous namespace\)::", "", r["Name"]); nm = nm[:nm.index("(")] if "(" in nm else nm
    print(f"{nm.replace('void ', ''):42s} calls {int(r['Calls']):4d}  avg {float(r['AverageNs'])/1e3:7.1f} us  {float(r['Percentage']):5.2f} %")
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_all.log 2>&1; rc=$?
tail -2 $O/tests_all.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_all.log | head -40; exit $rc; }
