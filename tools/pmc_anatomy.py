"""Per (kernel, grid) wave-cycle anatomy from SQ counter passes (tools/gpu_pmc_sq.sh):
fractions of SQ_WAVE_CYCLES spent waiting (s_waitcnt / barrier), issue-stalled, issuing; MFMA busy
per SIMD-cycle. SQ_WAVE_CYCLES / WAIT / ACTIVE count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles
(MI355X_MICROARCH.md, cycle constants table).  python tools/pmc_anatomy.py gpurun_out/pmc_TAG_1 gpurun_out/pmc_TAG_2"""
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
            acc[(k, r.get("Grid_Size", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), cs in acc.items():
    a = {c: sum(v) / len(v) for c, v in cs.items()}
    if "SQ_WAVE_CYCLES" not in a or a.get("SQ_INSTS_MFMA", a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)) == 0:
        continue
    w = a["SQ_WAVE_CYCLES"]
    busy = a.get("SQ_BUSY_CYCLES", 0)
    print(f"{k}  grid={g}")
    print(f"   wait(waitcnt/barrier) {a['SQ_WAIT_ANY'] / w:5.1%}  issue-stall {a['SQ_WAIT_INST_ANY'] / w:5.1%}  "
          f"issuing {a['SQ_ACTIVE_INST_ANY'] / w:5.1%}  (valu {a['SQ_ACTIVE_INST_VALU'] / w:5.1%}, "
          f"lds-stall {a.get('SQ_WAIT_INST_LDS', 0) / w:5.1%})")
    if busy:
        print(f"   MFMA busy / (SQ busy cycles x 4 SIMD x ...): {a['SQ_VALU_MFMA_BUSY_CYCLES']:.3g} cyc; SQ_BUSY {busy:.3g}")
    if a.get("SQ_INSTS_MFMA"):
        print(f"   VALU instructions per MFMA {a.get('SQ_INSTS_VALU', 0) / a['SQ_INSTS_MFMA']:.2f}")
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
        if c in a:
            print(f"   {c:22s} {a[c]:.4g}")
