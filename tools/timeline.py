"""Per-step GPU busy fraction and idle gaps from a rocprofv3 kernel_trace.csv (steps delimited
by the AdamW launch)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ad = [s for s, e, n in iv if "adamw" in n]
for a, b in zip(ad[:-1], ad[1:]):
    seg = sorted((max(s, a), min(e, b)) for s, e, n in iv if e > a and s < b)
    busy, gaps = 0, []
    cs, ce = seg[0]
    for s, e in seg[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce) / 1e3)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print("step %.2f ms  busy %.2f ms (%.1f%%)  gaps>20us: %s" % ((b - a) / 1e6, busy / 1e6, 100 * busy / (b - a),
                                                              [round(g) for g in gaps if g > 20][:12]))
