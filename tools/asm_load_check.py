"""Check that no instruction touches the destination VGPRs of an inline-asm register load
(`global_load_dwordx4` issued from asm, invisible to the compiler's waitcnt pass) before the
next `s_waitcnt vmcnt`, inside the loops of the selected kernels. A read there would see stale
data (the compiler believes the asm output is ready at once); a write would be clobbered.
Linear scan of the code before the first loop and of each loop body (the pending set carried
once around the back edge).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form --cuda-device-only \
        -S csrc/patch_embed.hip -o /tmp/pe.s
    python tools/asm_load_check.py /tmp/pe.s patch_fwd
"""
import re
import sys

from loop_waits import kernels


def vregs(op):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", op):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", op):
        out.add(int(m.group(1)))
    return out


def scan(seg, pending, bad, lab):
    for k, x in enumerate(seg):
        if not x or x[0] in ";.":
            continue
        if x.startswith("s_waitcnt") and "vmcnt" in x:
            pending.clear()
            continue
        op, _, args = x.partition(" ")
        if op.startswith("global_load_dwordx4"):
            for r in vregs(args.split(",")[0]):
                pending[r] = k
            continue
        dst, _, src = args.partition(",")
        touched = (vregs(src) | vregs(dst)) & set(pending)
        if touched and not op.startswith(("s_", "global_load_lds")):
            bad.append((lab, k, x))


def check(body):
    bad = []
    first = min([i for i, l in enumerate(body) if "Loop Header" in l] or [len(body)])
    scan([x.strip() for x in body[:first]], {}, bad, "prologue")
    heads = {l.split(":")[0].strip(): i for i, l in enumerate(body) if "Loop Header" in l}
    for lab, i in heads.items():
        ends = [k for k, x in enumerate(body) if re.search(r"s_c?branch\S*\s+" + re.escape(lab) + r"\s*$", x)]
        if not ends:
            continue
        seg = [x.strip() for x in body[i:max(ends) + 1]]
        pending = {}
        for _ in range(2):  # second pass: loads issued late in the body reach the top of the next trip
            scan(seg, pending, bad, lab)
    return bad


def main():
    path, sub = sys.argv[1], sys.argv[2]
    n = 0
    for name, body in kernels(path):
        if sub not in name:
            continue
        bad = check(body)
        n += len(bad)
        print(f"{len(bad):3d} early touches of asm-loaded registers  {name}")
        for b in bad[:10]:
            print("     ", b)
    sys.exit(1 if n else 0)


if __name__ == "__main__":
    main()
