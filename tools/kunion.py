"""Device time per launch of a kernel pair from a rocprofv3 kernel trace, counted the way bench.py's
roofline counts it: the union of the execution intervals of the matching kernels (both ViT streams'
launches overlap each other under the profiler as in the bench) / the number of launches of the
first kernel. The per-kernel averages in run_kernel_stats.csv sum each kernel's own interval, so
where two launches overlap they count the shared stretch twice.

    python tools/kunion.py gpurun_out/prof_TAG/run_kernel_trace.csv attn_bwd_dq_v3 attn_bwd_dkv_v3
"""
import csv
import sys


def main():
    path, names = sys.argv[1], sys.argv[2:]
    iv, n_first, own = [], 0, 0
    with open(path) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"]
            if any(n in k for n in names):
                s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                iv.append((s, e))
                own += e - s
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
    print(f"kernels {names}: {len(iv)} dispatches, {n_first} launches; union {tot / 1e6:.3f} ms "
          f"= {tot / max(n_first, 1) / 1e3:.1f} us per launch; sum of own intervals "
          f"{own / max(n_first, 1) / 1e3:.1f} us per launch")


if __name__ == "__main__":
    main()
