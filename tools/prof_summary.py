"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total/avg time and share."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r["Name"].replace("(anonymous namespace)::", "")[:100]
    print(f'{float(r["TotalDurationNs"]) / 1e6 / steps:8.2f} ms/step {100 * float(r["TotalDurationNs"]) / tot:5.1f}%  '
          f'calls/step {int(r["Calls"]) / steps:6.1f}  avg {float(r["AverageNs"]) / 1e3:8.1f} us  {n}')
print(f"total {tot / 1e6 / steps:.2f} ms/step")
