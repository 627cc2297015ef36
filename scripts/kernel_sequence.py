"""One training iteration's kernel sequence from a rocprofv3 --kernel-trace
CSV: the dispatches after the second-to-last solver-tail kernel
(k_fused_update_fail_batched) up to and including the last one.
Usage: kernel_sequence.py TRACE_DIR LABEL"""
import csv
import glob
import sys

d, label = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = [i for i, r in enumerate(rows) if "k_fused_update_fail_batched" in r["Kernel_Name"]]
if len(tail) < 2:
    sys.exit("fewer than two solver tails in the trace")
seq = rows[tail[-2] + 1:tail[-1] + 1]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seq]
print(f"{label} {len(seq)} kernels {sum(dur):.1f} us (profiled)")
for r, t in zip(seq, dur):
    name = r["Kernel_Name"].replace("void ", "").replace("rram::(anonymous namespace)::", "")
    grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    print(f"  {t:7.1f} us  grid {grid:>8}  {name[:90]}")
