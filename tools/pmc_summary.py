"""Summarise a rocprofv3 counter_collection.csv: one line per dispatch (kernel, counters),
skipping torch helper kernels (fills, random init)."""
import csv, sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
by = OrderedDict()
for r in rows:
    d = by.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "c": {}})
    d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, d in by.items():
    n = d["name"].replace("(anonymous namespace)::", "")
    if "at::native" in n or "rocclr" in n:
        continue
    cs = "  ".join(f"{c}={v:.4g}" for c, v in sorted(d["c"].items()))
    print(f"{k:>5} {n[:48]:48s} {cs}")
