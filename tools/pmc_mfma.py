"""MFMA utilisation per kernel from rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE CSVs.

SQ_VALU_MFMA_BUSY_CYCLES sums the matrix-core cycles of every MFMA of the dispatch over the chip
(= 16 x N for v_mfma_f32_16x16x32_bf16, 32 x N for 32x32x16; MI355X_MICROARCH.md PMC units);
GRBM_GUI_ACTIVE / 8 is the dispatch's cycles (rocprofv3 sums the 8 XCDs; it reads high on
dispatches shorter than ~0.3 ms).  busy = MFMA cycles / (dispatch cycles x 1024 SIMDs); the
effective clock = GRBM_GUI_ACTIVE / 8 / wall time.  Output: JSON per kernel (means over dispatches).
usage: pmc_mfma.py TAG csv...
"""

import collections
import csv
import json
import re
import sys

SIMDS = 256 * 4


def kname(n):
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", n)
    return m.group(0) if m else n[:80]


def main(tag, paths):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counters
    for p in paths:
        for r in csv.DictReader(open(p)):
            d = per[kname(r["Kernel_Name"])][(p, r["Dispatch_Id"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {"tag": tag, "definition": __doc__.strip().splitlines()[0], "kernels": {}}
    for k, ds in per.items():
        rows = [d for d in ds.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d]
        if not rows:
            continue
        busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in rows) / len(rows)
        cyc = sum(d["GRBM_GUI_ACTIVE"] / 8 for d in rows) / len(rows)
        ns = sum(d["ns"] for d in rows) / len(rows)
        if busy <= 0:
            continue
        out["kernels"][k] = {"dispatches": len(rows), "avg_us": round(ns / 1e3, 2),
                             "mfma_busy_cycles": busy, "dispatch_cycles": cyc,
                             "effective_clock_ghz": round(cyc / ns, 3) if ns else None,
                             "mfma_busy": round(busy / (cyc * SIMDS), 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
