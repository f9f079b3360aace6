"""Check that M0 is only written by ivit_common.h's glds<> sequence in the emitted device code.

glds<> sets M0 in inline asm that the compiler cannot see; this is safe only while no
compiler-generated instruction keeps a value in M0. Every line naming m0 must be the
`s_mov_b32 m0, sN` of that sequence, followed by `s_nop 0` and the global_load_lds.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/attention.hip -o /tmp/a.s
    python tools/check_m0.py /tmp/a.s [/tmp/b.s ...]
"""
import re
import sys


def check(path):
    lines = [l.split(";")[0].strip() for l in open(path)]
    bad = []
    for i, l in enumerate(lines):
        if not re.search(r"\bm0\b", l):
            continue
        ok = (re.match(r"s_mov_b32 m0, s\d+$", l) and lines[i + 1] == "s_nop 0"
              and lines[i + 2].startswith("global_load_lds_dword"))
        if not ok:
            bad.append((i + 1, l))
    return bad


if __name__ == "__main__":
    rc = 0
    for p in sys.argv[1:]:
        bad = check(p)
        print(p, "ok" if not bad else f"{len(bad)} foreign M0 uses")
        for ln, l in bad[:20]:
            print(f"  {ln}: {l}")
        rc |= bool(bad)
    sys.exit(rc)
