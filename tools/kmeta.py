"""Kernel resource summary from a device assembly file (hipcc --cuda-device-only -S):
LDS bytes, VGPR/AGPR counts and spills for kernels whose name contains a substring.

    python tools/kmeta.py attention.s attn_fwd
"""
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    s = open(path).read()
    m = s[s.index("amdhsa.kernels:"):]
    for b in m.split("\n  - "):
        name = re.search(r"\.name:\s+(\S+)", b)
        if not name or sub not in name.group(1):
            continue

        def g(k):
            r = re.search(r"\.%s:\s+(\S+)" % k, b)
            return r.group(1) if r else None
        print(f"{name.group(1)[:90]:90s} lds {g('group_segment_fixed_size')} vgpr {g('vgpr_count')} "
              f"agpr {g('agpr_count')} spill {g('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
