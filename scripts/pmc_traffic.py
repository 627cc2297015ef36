"""HBM traffic of the bench's dominant kernels from rocprofv3 --pmc passes
(scripts/pmc.sh output: one pass with FETCH_SIZE, one with WRITE_SIZE, over
`bench.py --steps 3 --warmup 1`).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores.

Per-launch traffic for the injection kernel; per-step traffic for the
conv/IP GEMM set (all k_gemm* / k_conv_* / k_splitk_reduce dispatches and
the x6 operand packs / forwards run), next to the algorithmic bytes of AlexNet b256's conv1-5 + fc6-8
(each layer's input activation + weights read once, output written once).
Writes JSON to stdout (bench.py reads the committed copy in profiles/)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
forwards = int(sys.argv[2]) if len(sys.argv) > 2 else 4   # 1 warmup + 3 timed steps
tot = defaultdict(float)       # (kernel class, counter) -> sum over dispatches
cnt = defaultdict(int)         # (kernel class, counter) -> dispatches
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name, c = r["Kernel_Name"], r["Counter_Name"]
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        if "k_inject_batched" in name:
            k = "inject"
        elif any(t in name for t in ("k_gemm", "k_conv_", "k_splitk_reduce", "k_pack_rows_x6", "k_pack_octets_x6")):
            # every kernel of the conv1-5 + fc6-8 contractions, their operand
            # packs (weights split per call, inputs split into octets) included
            k = "gemm"
        else:
            continue
        tot[(k, c)] += float(r["Counter_Value"])
        cnt[(k, c)] += 1
KIB = 1024.0
# AlexNet b256 (bvlc_alexnet TEST): (input elems, weight elems, output elems) per image-batch
B = 256
ALEX = [(3*227*227*B, 96*363, 96*55*55*B), (96*27*27*B, 256*48*25, 256*27*27*B),
        (256*13*13*B, 384*256*9, 384*13*13*B), (384*13*13*B, 384*192*9, 384*13*13*B),
        (384*13*13*B, 256*192*9, 256*13*13*B), (9216*B, 4096*9216, 4096*B),
        (4096*B, 4096*4096, 4096*B), (4096*B, 1000*4096, 1000*B)]
ALG_BYTES = 4.0 * sum(a + w + o for a, w, o in ALEX)
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 3 --warmup 1 ({root})",
       "correction": "bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950 FETCH_SIZE half-count)"}
if cnt[("inject", "FETCH_SIZE")] and cnt[("inject", "WRITE_SIZE")]:
    fb = 2 * KIB * tot[("inject", "FETCH_SIZE")] / cnt[("inject", "FETCH_SIZE")]
    wb = KIB * tot[("inject", "WRITE_SIZE")] / cnt[("inject", "WRITE_SIZE")]
    out["inject"] = {"bytes_per_launch": fb + wb, "read_bytes": fb, "write_bytes": wb,
                     "launches": cnt[("inject", "FETCH_SIZE")]}
if cnt[("gemm", "FETCH_SIZE")] and cnt[("gemm", "WRITE_SIZE")]:
    fb = 2 * KIB * tot[("gemm", "FETCH_SIZE")] / forwards
    wb = KIB * tot[("gemm", "WRITE_SIZE")] / forwards
    out["gemm"] = {"bytes_per_step": fb + wb, "read_bytes": fb, "write_bytes": wb,
                   "dispatches_per_step": cnt[("gemm", "FETCH_SIZE")] / forwards,
                   "algorithmic_bytes_per_step": ALG_BYTES,
                   "ratio_to_algorithmic": (fb + wb) / ALG_BYTES}
print(json.dumps(out, indent=1))
