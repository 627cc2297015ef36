"""Per-kernel averages of rocprofv3 --pmc counter CSVs (AlexNet MC kernels by short name).
Usage: pmc_kernels.py DIR [DIR ...]  (each DIR holds a run_counter_collection.csv tree)"""
import csv,glob,sys,collections
def load(d):
    tot=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.defaultdict(lambda: collections.defaultdict(int))
    for f in glob.glob(f"{d}/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(f)):
            k=r["Kernel_Name"]
            for pat,short in [("k_conv1_ring","conv1"),("cb16_x6ILi5","conv2"),("cb_x6ILi3ELi3ELi4ELi8","conv3"),("cb_x6ILi3ELi3ELi2ELi4","conv4"),("cb16_x6ILi3","conv5"),("k_gemm_x6","fc67"),("k_lrn_maxpool_band","lrnpool"),("k_inject","inject"),("k_gemm2","fc8")]:
                if pat in k:
                    tot[short][r["Counter_Name"]]+=float(r["Counter_Value"]); n[short][r["Counter_Name"]]+=1
    return tot,n
for d in sys.argv[1:]:
    tot,n=load(d)
    print(d)
    for k in tot:
        print("  %-8s"%k, " ".join("%s=%.3g"%(c,tot[k][c]/n[k][c]) for c in sorted(tot[k])))
