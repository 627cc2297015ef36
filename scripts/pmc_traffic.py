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
forwards = int(sys.argv[2]) if len(sys.argv) > 2 else 7   # 1 warmup + 3 timed + 3 contraction-table steps
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

# ---- per-kernel table: measured vs algorithmic bytes per step ----
# algorithmic bytes of each AlexNet b256 kernel in the operand form the engine
# reads (the bf16x6 kernels read pre-split octets: 6 B per element; fp32
# tensors 4 B), each tensor once; split-K partials and the packs' own outputs
# count as the bytes they must move
MB = 1e6
A1, Y1 = 3*227*227*B*4, 96*55*55*B*4
P1O, P1Y = 96*27*27*B*6, 96*27*27*B*4
Y2 = 256*27*27*B*4
P2O, P2Y = 256*13*13*B*6, 256*13*13*B*4
Y3 = Y4 = 384*13*13*B*4
O4 = 384*13*13*B*6
Y5 = 256*13*13*B*4
ALG = {  # class: (algorithmic bytes per step, description)
    "conv1 k_conv1_ring_x6": (A1 + 96*363*4 + Y1, "x fp32 + w + y"),
    # (round 5: the pooled fp32 y is materialised only on read -- the
    # pooled-output fold, conv2 / conv3 take the companion -- so not written)
    "norm1+pool1 (LRN + max pool, octets)": (Y1 + P1O, "x + y octets"),
    "conv2 k_conv_cb16_x6<5,5,...>": (P1O + 256*48*25*4 + Y2, "x octets + w + y"),
    "norm2+pool2 (LRN + max pool, octets)": (Y2 + P2O, "x + y octets"),
    "conv3 k_conv_cb16_x6<3,3,4,4,...>": (P2O + 384*256*9*4 + Y3, "x octets + w + y"),
    "conv4/conv5 input packs k_pack_octets_x6": (2 * (Y3 + O4), "2 x (read fp32, write octets)"),
    "conv4 k_conv_cb16_x6<3,3,2,2,...>": (O4 + 384*192*9*4 + Y4, "x octets + w + y"),
    "conv5 k_conv_cb16_x6<3,3,4,4,...>": (O4 + 256*192*9*4 + Y5, "x octets + w + y"),
    "fc6/fc7 k_gemm_x6 + k_pack_rows_x6": ((9216 + 4096)*B*(4 + 6 + 6) + (4096*9216 + 4096*4096)*4 + 2*4096*B*4,
                                            "x read + slabs written/read, w, y"),
    "fc8 k_gemm2": (4096*B*4 + 1000*4096*4 + 1000*B*4, "x + w + y"),
    "split-K reductions": (0.0, "partials (no algorithmic counterpart)"),
    "injection k_inject_batched": (8.0 * 58631144, "read clean + write faulted"),
}


def classify(name, grid=0):
    if "k_inject_batched" in name:
        return "injection k_inject_batched"
    if "k_conv1_ring_x6" in name:
        return "conv1 k_conv1_ring_x6"
    if "lrn_maxpool" in name:
        return None  # split below by grid
    # (k_conv_cb16_x6: the 16x16x32 form of the same kernel, round 4)
    name = name.replace("k_conv_cb16_x6", "k_conv_cb_x6")
    if "k_conv_cb_x6ILi5ELi5" in name or "k_conv_cb_x6<5, 5" in name:
        return "conv2 k_conv_cb16_x6<5,5,...>"
    if "k_conv_cb_x6ILi3ELi3ELi4ELi8" in name:
        return "conv3 k_conv_cb16_x6<3,3,4,4,...>"
    if "k_conv_cb_x6ILi3ELi3ELi2ELi" in name:
        return "conv4 k_conv_cb16_x6<3,3,2,2,...>"
    if "k_conv_cb_x6ILi3ELi3ELi4ELi4" in name:
        # round 5: conv3 and conv5 both run the 128 x 128 16x16x32 form; conv3's
        # grid is the larger (3 x 338 vs 2 x 338 workgroups)
        return "conv3 k_conv_cb16_x6<3,3,4,4,...>" if grid > 200000 else "conv5 k_conv_cb16_x6<3,3,4,4,...>"
    if "k_pack_octets_x6" in name:
        return "conv4/conv5 input packs k_pack_octets_x6"
    if "k_gemm_x6" in name or "k_pack_rows_x6" in name:
        return "fc6/fc7 k_gemm_x6 + k_pack_rows_x6"
    if "k_gemm2" in name:
        return "fc8 k_gemm2"
    if "k_splitk_reduce" in name:
        return "split-K reductions"
    # once per process, not per map: the runtime's fills / copies (net setup,
    # the MC driver's clean weight copies), the synthetic data and filler
    # kernels, the weight packs (cached across maps after the first)
    if any(t in name for t in ("__amd_rocclr", "k_fill", "k_set", "_pack_x6", "at::native")):
        return "setup"
    return "other"


per = defaultdict(float)
lrn_grids = {}
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name, c = r["Kernel_Name"], r["Counter_Name"]
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        k = classify(name, int(r.get("Grid_Size", 0) or 0))
        if k is None:
            lrn_grids.setdefault(int(r["Grid_Size"]), []).append((c, float(r["Counter_Value"])))
            continue
        per[k] += (2 if c == "FETCH_SIZE" else 1) * KIB * float(r["Counter_Value"])
# the two LRN + pool launches: the larger grid is norm1 / pool1 (96 x 55 x 55 input)
for i, (gsz, vals) in enumerate(sorted(lrn_grids.items(), reverse=True)):
    k = "norm1+pool1 (LRN + max pool, octets)" if i == 0 else "norm2+pool2 (LRN + max pool, octets)"
    per[k] += sum((2 if c == "FETCH_SIZE" else 1) * KIB * v for c, v in vals)
# octet companions from the convolution epilogues (RRAM_OCTETS=1, the default
# since round 3): conv3 / conv4 write their outputs' companions and no input
# pack runs, so those bytes move from the pack row to the producers' rows
# (round 6: the TEST-phase convolution-output fold -- conv3 / conv4 are read
# only by conv4 / conv5 through the companion -- writes no fp32 y for them)
if per.get("conv4/conv5 input packs k_pack_octets_x6", 0.0) == 0.0:
    ALG["conv3 k_conv_cb16_x6<3,3,4,4,...>"] = (P2O + 384*256*9*4 + O4, "x octets + w + y octets (y fp32 folded)")
    ALG["conv4 k_conv_cb16_x6<3,3,2,2,...>"] = (O4 + 384*192*9*4 + O4, "x octets + w + y octets (y fp32 folded)")
    ALG["conv4/conv5 input packs k_pack_octets_x6"] = (0.0, "none run (companions from the conv3 / conv4 epilogues)")
table = {}
for k, (alg, what) in ALG.items():
    meas = per.get(k, 0.0) / forwards
    table[k] = {"measured_MB_per_step": round(meas / MB, 1), "algorithmic_MB_per_step": round(alg / MB, 1),
                "ratio": round(meas / alg, 3) if alg else None, "algorithmic": what}
if per.get("other"):
    table["other"] = {"measured_MB_per_step": round(per["other"] / forwards / MB, 1),
                      "what": "every other per-map kernel (pool5, softmax, accuracy, MC statistics)"}
if per.get("setup"):
    table["setup (not per map)"] = {"measured_MB_total": round(per["setup"] / MB, 1),
                                    "what": "runtime fills / copies, data and filler kernels, first-map weight packs"}
out["per_kernel"] = table
print(json.dumps(out, indent=1))
