"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel into a JSON table.

    python tools/pmc_summary.py gpurun_out/pmcf_TAG gpurun_out/pmcw_TAG > profiles/rNN_pmc_hbm.json

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced (16 B/lane) streaming reads, so the
read bytes are 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane stores.
Every kernel on the hot path reads with 16-B lanes (global_load_lds / uint4 loads).
"""
import csv
import glob
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
                acc[row["Kernel_Name"]].append((float(row["Counter_Value"]), dur))
    return acc


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
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
    json.dump({"source": [fdir, wdir], "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950), write = WRITE_SIZE KiB x 1024",
               "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
