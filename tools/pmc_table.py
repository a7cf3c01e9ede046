"""Pivot rocprofv3 --pmc counter_collection CSVs into one row per (kernel, dispatch)."""
import csv, re, sys, collections
rows = collections.OrderedDict()
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void dh::", "")
        key = (name, r.get("Grid_Size", ""), r.get("Dispatch_Id", ""))
        rows.setdefault((name, r.get("Grid_Size", "")), collections.defaultdict(list))[r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, grid), cnt in rows.items():
    print(name, "grid", grid, {k: f"{sum(v)/len(v):.4g}" for k, v in cnt.items()})
