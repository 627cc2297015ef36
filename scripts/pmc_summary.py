"""Summarise rocprofv3 --pmc CSVs (scripts/pmc.sh output): per kernel name (shortened)
and grid size, mean of each counter over dispatches."""
import csv
import glob
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        m = re.search(r"k_(gemm2?|conv_patch(?:_x6)?)<([^>]*)>", name)
        if m:
            short = f"{m.group(1)}<" + m.group(2).replace(" ", "") + ">"
        else:
            short = re.sub(r"\(anonymous namespace\)::", "", name)
            short = re.sub(r"\(.*", "", short).replace("void ", "").split("::")[-1][:40]
        key = (short, r["Grid_Size"])
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cols = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
        "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
        "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VMEM_RD", "GRBM_GUI_ACTIVE", "FETCH_SIZE",
        "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"]
for key in sorted(agg, key=lambda k: -sum(dur[k]) / max(len(dur[k]), 1)):
    d = agg[key]
    us = sorted(dur[key])[len(dur[key]) // 2]
    if us < 5:
        continue
    vals = " ".join(f"{c}={sum(d[c]) / len(d[c]):.3g}" for c in cols if c in d)
    print(f"{key[0]:>28s} grid={key[1]:>9s} ~{us:8.1f}us  {vals}")
