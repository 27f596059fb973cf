"""Per-kernel time per step from a rocprofv3 --stats kernel_stats.csv: python tools/kstats.py FILE STEPS [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time per step {tot / steps / 1e6:.2f} ms ({steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:9.2f} ms/step  {int(r['Calls']) / steps:7.1f}/step  "
          f"avg {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
