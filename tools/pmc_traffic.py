"""HBM traffic per GEMM launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs.

Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts 64 B per 128-B request of a
wide (16 B / lane) streaming read -> doubled (the GEMMs stage both operands with 16-B
LDS-DMA); WRITE_SIZE is taken as is.  Both counters are in KiB.  Output: JSON with
per-kernel and aggregate bytes per launch over all GEMM dispatches (log-psi + channel).
"""

import collections
import csv
import json
import re
import sys


def kname(n):
    m = re.search(r"(gemm\w*_kernel)(<[^>]*>)?", n)
    return m.group(0) if m else n[:80]


def main(paths):
    per = collections.defaultdict(lambda: {"FETCH_SIZE": [], "WRITE_SIZE": []})
    for p in paths:
        for r in csv.DictReader(open(p)):
            c = r["Counter_Name"]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                per[kname(r["Kernel_Name"])][c].append(float(r["Counter_Value"]) * 1024.0)
    out = {"correction": "FETCH_SIZE x2 (wide 16-B reads), WRITE_SIZE x1; KiB -> bytes", "kernels": {}}
    tot_b = tot_n = 0.0
    for k, v in per.items():
        nf, nw = len(v["FETCH_SIZE"]), len(v["WRITE_SIZE"])
        if not nf or not nw:
            continue
        rd = 2.0 * sum(v["FETCH_SIZE"]) / nf
        wr = sum(v["WRITE_SIZE"]) / nw
        out["kernels"][k] = {"launches": nf, "read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
        tot_b += (rd + wr) * nf
        tot_n += nf
    out["gemm_bytes_per_launch"] = tot_b / tot_n if tot_n else None
    # the local-energy channel GEMMs alone (split-bf16 kernel families, incl. the fused
    # GEMM + channel LayerNorm of gemm_lnch.hip; not its MODE 2, layer 1 whole: bench.py's
    # roofline class is the 256-deep maps)
    ch = [v for k, v in out["kernels"].items() if k.startswith(("gemm_x6q_kernel", "gemm_x6m_kernel", "gemm_lnch_kernel"))
          and not re.match(r"gemm_lnch_kernel<\d+, 2", k)]
    n_ch = sum(v["launches"] for v in ch)
    out["channel_gemm_bytes_per_launch"] = (
        sum(v["bytes_per_launch"] * v["launches"] for v in ch) / n_ch if n_ch else None)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
