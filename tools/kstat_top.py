"""Per-step kernel time summary of a rocprofv3 --stats run: python tools/kstat_top.py <kernel_stats.csv> [steps] [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel ms per step: {tot / steps / 1e6:.3f}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step  calls/step {int(r['Calls']) / steps:6.1f}  "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")
