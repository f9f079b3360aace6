"""List the compiler-inserted `s_waitcnt vmcnt` inside the loops of selected kernels.

Kernels that stream tiles with the inline-asm LDS DMA (ivit_common.h glds<>) retire them with
their own counted waits. A compiler wait inside such a loop (e.g. at the first in-loop use of a
register that was loaded before the loop) also waits for the in-flight DMA of the next tile,
so every one found here serialises the prefetch.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/attention.hip -o /tmp/a.s
    python tools/loop_waits.py /tmp/a.s attn_bwd gemm_bf16_glds
"""
import re
import sys


def kernels(path):
    s = open(path).read().split("\n")
    starts = [i for i, l in enumerate(s) if re.match(r"^_Z\S*:", l)]
    for a, b in zip(starts, starts[1:] + [len(s)]):
        yield s[a].split(":")[0], s[a:b]


def loop_waits(body):
    out = []
    heads = {l.split(":")[0].strip(): i for i, l in enumerate(body) if "Loop Header" in l}
    for lab, i in heads.items():
        ends = [k for k, x in enumerate(body) if re.search(r"s_c?branch\S*\s+" + re.escape(lab) + r"\s*$", x)]
        if not ends:
            continue
        in_asm = False
        for k in range(i, max(ends) + 1):
            x = body[k].strip()
            if x.startswith(";;#ASMSTART"):
                in_asm = True
            elif x.startswith(";;#ASMEND"):
                in_asm = False
            elif not in_asm and x.startswith("s_waitcnt") and "vmcnt" in x:
                out.append((lab, k, x))
    return out


if __name__ == "__main__":
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if subs and not any(s in name for s in subs):
            continue
        w = loop_waits(body)
        print(f"{len(w):3d} compiler vmcnt waits in loops  {name[:110]}")
        for lab, k, x in w[:8]:
            print(f"      {lab} +{k}: {x}")
