"""Register / spill / scratch / LDS summary of the kernels in a hipcc -S assembly file.
Usage: python tools/kres.py file.s [name-regex]"""
import re
import sys

txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for blk in txt.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name:
        continue
    n = name.group(1)
    if pat and not pat.search(n):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]  # noqa: E731
    short = re.sub(r"_ZN2dh12_GLOBAL__N_1\d+", "", n)[:60]
    print(f"{short:60s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>4} "
          f"scratch {g('private_segment_fixed_size'):>5} lds {g('group_segment_fixed_size'):>6}")
