#!/bin/bash
# Iteration check on one box: a subset of the GPU tests ($TESTS, default the
# layer / octet / host files), a kernel trace of the headline bench (the
# per-kernel averages of $SHOW kernels), FETCH / WRITE PMC passes -> the
# per-kernel traffic table.  Usage: TESTS="tests/x.py -k y" SHOW="lrn|conv" scripts/gpu_check.sh
set -o pipefail
R=$(pwd); O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_layers.py tests/test_gpu_octets.py tests/test_gpu_host.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_chk.log 2>&1; rc=$?
tail -1 $O/pytest_chk.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/pytest_chk.log | head -20; exit $rc; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_chk -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/$O/bench_chk.json 2> $R/$O/bench_chk.err ) || { tail -5 $O/bench_chk.err; exit 1; }
python3 - $O/prof_chk/run_kernel_stats.csv $O/bench_chk.json "${SHOW:-lrn|accuracy}" <<'PY'
import csv, json, re, sys
d = json.load(open(sys.argv[2]))
print(d["value"], d["ms_per_step"], "roofline", d["roofline"]["achieved"], d["roofline"]["frac"], d["roofline"]["avg_us_per_launch"])
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        print("  ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/$O/pmc_chk/p_$c -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_chk_$c.log 2>&1 ) || { echo "pmc $c failed"; tail -5 $O/pmc_chk_$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py $O/pmc_chk > $O/pmc_chk_traffic.json && python3 -c "
import json; d=json.load(open('$O/pmc_chk_traffic.json'))
for k,v in d['per_kernel'].items(): print(k, v)"
