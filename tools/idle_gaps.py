"""GPU idle time inside one training step of a rocprofv3 kernel trace: the step is the stretch
between the last two FusedAdamW launches; a gap is time when no kernel runs on any stream. Prints
the step span, the total idle time and the largest gaps with the kernels either side.

    python tools/idle_gaps.py <run_kernel_trace.csv> [n_gaps]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r["Stream_Id"])
                for r in rows)
    ad = [i for i, k in enumerate(ks) if "adamw" in k[2].lower()]
    if len(ad) < 2:
        sys.exit("need two optimizer launches in the trace")
    seg = ks[ad[-2] + 1:ad[-1] + 1]
    t0, t1 = seg[0][0], max(k[1] for k in seg)
    gaps, end, prev = [], seg[0][1], seg[0]
    for k in seg[1:]:
        if k[0] > end:
            gaps.append(((k[0] - end) / 1e3, (k[0] - t0) / 1e6, prev, k))
        if k[1] > end:
            end, prev = k[1], k
    print(f"step span {(t1 - t0) / 1e6:.3f} ms, {len(seg)} kernels, idle {sum(g[0] for g in gaps):.1f} us "
          f"in {len(gaps)} gaps")
    for us, at, a, b in sorted(gaps, reverse=True)[:top]:
        print(f"{us:7.1f} us at {at:7.3f} ms | s{a[3]} {a[2]} -> s{b[3]} {b[2]}")


if __name__ == "__main__":
    main()
