"""Per-launch average of the LRN + max pool band kernels in a rocprofv3 output
directory: kernel-trace duration (us) or the FETCH_SIZE counter (bytes,
doubled per the gfx950 correction).  Usage: lrn_stats.py DIR LABEL"""
import csv
import glob
import sys
from collections import defaultdict

d, label = sys.argv[1], sys.argv[2]
acc = defaultdict(list)
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "lrn_maxpool_band" in n:
            acc[n.split("<")[1].split(">")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "lrn_maxpool_band" in n and r["Counter_Name"] == "FETCH_SIZE":
            acc[n.split("<")[1].split(">")[0] + " FETCH MB"].append(2 * 1024 * float(r["Counter_Value"]) / 1e6)
for k, v in sorted(acc.items()):
    v = v[len(v) // 4:]  # drop the warmup launches
    print(f"[{label}] {k}: {sum(v) / len(v):.1f} over {len(v)}", flush=True)
