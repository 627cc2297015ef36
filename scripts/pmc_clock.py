"""Per-kernel effective clock and MFMA-busy fraction from a pmc_summary.py
listing (MI355X_MICROARCH.md 'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 /
wall; busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / those cycles)."""
import re
import sys

for line in open(sys.argv[1]):
    m = re.match(r"\s*(\S+) grid=\s*(\d+) ~\s*([\d.]+)us(.*)", line)
    if not m:
        continue
    d = {k: float(v) for k, v in re.findall(r"(\w+)=([\d.e+]+)", m.group(4))}
    us = float(m.group(3))
    cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8
    if us < 20 or not cyc:
        continue
    wave = d.get("SQ_WAVE_CYCLES", 1)
    print(f"{m.group(1):32s} grid={m.group(2):>8s} {us:8.1f}us clk={cyc / us / 1e3:.2f}GHz "
          f"mfma_busy={d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / cyc:.2f} "
          f"wait_any={d.get('SQ_WAIT_ANY', 0) / wave:.2f} wait_inst={d.get('SQ_WAIT_INST_ANY', 0) / wave:.2f}")
