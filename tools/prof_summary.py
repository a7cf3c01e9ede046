"""Condense a rocprofv3 --stats kernel CSV into a markdown table (profiles/*.md)."""

import csv
import re
import sys


def short(name):
    m = re.search(r"dh::\(anonymous namespace\)::(\w+(<[^>]*>)?)", name)
    if m:
        return m.group(1)
    if name.startswith("Cijk"):
        return "hipBLASLt Cijk (parameter packing, untimed)"
    m = re.search(r"at::native::(\w+)", name)
    return f"torch {m.group(1)}" if m else name[:60]


def main(path, title):
    rows = list(csv.DictReader(open(path)))
    print(f"# {title}\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        print(
            f"| {short(r['Name'])} | {r['Calls']} | {int(r['TotalDurationNs']) / 1e6:.3f} | "
            f"{float(r['AverageNs']) / 1e3:.2f} | {int(r['MinNs']) / 1e3:.2f} | {int(r['MaxNs']) / 1e3:.2f} | "
            f"{float(r['Percentage']):.2f} |"
        )


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "rocprofv3 kernel stats")
