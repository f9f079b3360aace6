"""Summarise a rocprofv3 kernel_stats.csv: per-kernel ms per step (divide by --steps)."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    n = r['Name'].replace('(anonymous namespace)::', '').replace('_ZN4ivit16gemm_bf16_kernelI', 'gemm<')
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step {float(r['Percentage']):5.1f}% calls={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {n[:110]}")
print(f'total {tot/1e6/steps:.2f} ms/step')
