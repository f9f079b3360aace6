"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel into a JSON table.

    python tools/pmc_summary.py gpurun_out/pmcf_TAG gpurun_out/pmcw_TAG [REGEX] > profiles/rNN_pmc_hbm.json

REGEX: kernels whose name matches it are also listed per launch (dispatch order; the FETCH and
WRITE runs launch the same sequence) and split into a "large" and a "small" class at the
geometric mean of their extreme read sizes — e.g. the LiDAR (290-channel) and map (9-channel)
launches of one kernel, whose raster bytes differ ~30x.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced (16 B/lane) streaming reads, so the
read bytes are 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane stores.
Every kernel on the hot path reads with 16-B lanes (global_load_lds / uint4 loads).
"""
import csv
import glob
import math
import re
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name
    for pre in ("void ", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n.split("(")[0][:160]


def load(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                acc[row["Kernel_Name"]].append((int(row.get("Dispatch_Id", 0) or 0), float(row["Counter_Value"]), dur))
    for k in acc:
        acc[k] = [(v, d) for _, v, d in sorted(acc[k])]
    return acc


def per_launch(f, w):
    rows = []
    for i, (fv, dur) in enumerate(f):
        wv = w[i][0] if i < len(w) else None
        rows.append({"launch": i, "read_bytes": 2 * fv * 1024, "write_bytes": wv * 1024 if wv is not None else None,
                     "dur_us": dur / 1e3})
    out = {"launches": rows}
    if len(rows) >= 2:
        lo, hi = min(r["read_bytes"] for r in rows), max(r["read_bytes"] for r in rows)
        if lo > 0 and hi / lo > 4:
            cut = math.sqrt(lo * hi)
            for cls, sel in (("large", lambda r: r["read_bytes"] >= cut), ("small", lambda r: r["read_bytes"] < cut)):
                rs = [r for r in rows if sel(r)]
                out[cls] = {"launches": len(rs),
                            "read_bytes_avg": sum(r["read_bytes"] for r in rs) / len(rs),
                            "write_bytes_avg": (sum(r["write_bytes"] or 0 for r in rs) / len(rs)),
                            "dur_us_avg": sum(r["dur_us"] for r in rs) / len(rs)}
    return out


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write), key=lambda k: -sum(v for v, _ in fetch.get(k, [])) * 2):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(v for v, _ in f) / len(f) if f else None
        wk = sum(v for v, _ in w) / len(w) if w else None
        rd = 2 * fk * 1024 if fk is not None else None
        wr = wk * 1024 if wk is not None else None
        out[short(k)] = {
            "launches": len(f), "fetch_size_kib_avg": fk, "write_size_kib_avg": wk,
            "hbm_read_bytes_avg": rd, "hbm_write_bytes_avg": wr,
            "hbm_bytes_avg": (rd or 0) + (wr or 0) if (rd is not None or wr is not None) else None,
            "full_name": k,
        }
        if rx is not None and rx.search(k):
            out[short(k)]["per_launch"] = per_launch(f, w)
    json.dump({"source": [fdir, wdir], "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950), write = WRITE_SIZE KiB x 1024",
               "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
