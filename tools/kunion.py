"""Device time per launch of a kernel pair from a kernel-interval CSV, counted the way bench.py's
roofline counts it: the union of the execution intervals of the matching kernels (both ViT streams'
launches overlap each other) / the number of launches of the first kernel. The per-kernel averages
in run_kernel_stats.csv sum each kernel's own interval, so where two launches overlap they count the
shared stretch twice.

Inputs (same columns, Kernel_Name / Start_Timestamp / End_Timestamp in ns):
  * a rocprofv3 kernel trace (run_kernel_trace.csv of a profiled bench command), or
  * the intervals bench.py recorded in its own timed region (bench.py --intervals-out: the HIP
    event pairs bound to each attention launch, the source of the line's roofline.frac).

    python tools/kunion.py TRACE.csv attn_bwd_dq_v3 attn_bwd_dkv_v3 [--flops F] [--json OUT]

--flops: algorithmic flop per launch (bench.py attn_flops) -> TFLOP/s and the fraction of the
dense bf16 MFMA peak; --json: write the summary (bench.py reads the newest committed
profiles/*_attn_bwd_union.json of kind rocprofv3 into roofline.frac_rocprof, only when the kernel
names it matched are the kernels the entry point launches now, and names the file and its time).
"""
import argparse
import csv
import json
import time

PEAK_BF16_TFLOPS = 2516.6


def union(path, names):
    iv, n_first, own, matched = [], 0, 0, set()
    with open(path) as fh:
        rows = csv.DictReader(fh)
        kind = "bench_intervals" if "Launch" in (rows.fieldnames or []) else "rocprofv3"
        for row in rows:
            k = row["Kernel_Name"]
            if any(n in k for n in names):
                s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                iv.append((s, e))
                own += e - s
                matched.add(k)
                if names[0] in k:
                    n_first += 1
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return {"source": path, "source_kind": kind, "kernels": names, "kernel_names": sorted(matched),
            "generated_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "dispatches": len(iv), "launches": n_first,
            "union_ms": tot / 1e6, "union_us_per_launch": tot / max(n_first, 1) / 1e3,
            "own_us_per_launch": own / max(n_first, 1) / 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("names", nargs="+")
    ap.add_argument("--flops", type=float, default=None)
    ap.add_argument("--json", type=str, default=None)
    a = ap.parse_args()
    d = union(a.path, a.names)
    print(f"kernels {d['kernels']}: {d['dispatches']} dispatches, {d['launches']} launches; union "
          f"{d['union_ms']:.3f} ms = {d['union_us_per_launch']:.1f} us per launch; sum of own intervals "
          f"{d['own_us_per_launch']:.1f} us per launch")
    if a.flops:
        tf = a.flops / (d["union_us_per_launch"] * 1e-6) / 1e12
        d.update(flops_per_launch=a.flops, tflops=round(tf, 2), frac=round(tf / PEAK_BF16_TFLOPS, 4),
                 peak_tflops=PEAK_BF16_TFLOPS)
        print(f"{a.flops:.4g} flop per launch: {tf:.1f} TFLOP/s = {tf / PEAK_BF16_TFLOPS:.4f} of {PEAK_BF16_TFLOPS}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(d, fh, indent=1)


if __name__ == "__main__":
    main()
