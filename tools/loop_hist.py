"""Instruction histogram of each loop body (loop header .. back edge) of the selected kernels in
a device assembly file — a static view of what one trip issues (v_mov shuffles, readlane
spills, conversions, waits).   python tools/loop_hist.py file.s kernel_substring [top]"""
import re
import sys
from collections import Counter

from loop_waits import kernels


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    for name, body in kernels(path):
        if sub not in name:
            continue
        heads = [(i, l.split(":")[0].strip()) for i, l in enumerate(body) if "Loop Header" in l]
        for i, lab in heads:
            ends = [k for k, x in enumerate(body) if re.search(r"s_c?branch\S*\s+" + re.escape(lab) + r"\s*$", x)]
            if not ends:
                continue
            ins = [x.split()[0] for x in body[i:max(ends) + 1]
                   if x.strip() and not x.strip().startswith((";", ".")) and not x.startswith("\t;")]
            c = Counter(ins)
            mf = sum(v for k, v in c.items() if "mfma" in k)
            valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
            print(f"{name[:70]} {lab}: {len(ins)} instr, {mf} mfma, {valu} valu")
            for k, v in c.most_common(top):
                print(f"   {v:5d} {k}")


if __name__ == "__main__":
    main()
