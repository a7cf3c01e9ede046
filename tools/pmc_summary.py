"""Summarise rocprofv3 --pmc CSVs of one kernel: duration, clock, MFMA busy, wait shares.

usage: python tools/pmc_summary.py gpurun_out/pmcg/v200 [more dirs]
Clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES
over 1024 SIMDs x those cycles."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    vals = collections.defaultdict(list)
    durs = []
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not durs:
        print(d, "no data")
        continue
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    dur = sorted(durs)[len(durs) // 2]
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    out = [f"{d}: {dur:.1f} us"]
    if cyc:
        out.append(f"clk {cyc / dur / 1e3:.2f} GHz")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and cyc:
        out.append(f"mfma busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.1%}")
    if "SQ_INSTS_MFMA" in m:
        mf = m["SQ_INSTS_MFMA"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if k in m:
                out.append(f"{k[9:]}/mfma {m[k] / mf:.2f}")
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in m:
                out.append(f"{k[3:]} {m[k] / wc:.0%}")
    if "TCC_HIT_sum" in m:
        out.append(f"L2 hit {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.0%}")
    print("  ".join(out))
