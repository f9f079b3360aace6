"""ASan host build of the C ABI's argument validation, workspace queries and host-side bookkeeping
(SURVEY.md §5 sanitizers: host code only — GPU ASan is not available on this pool).

Compiles every csrc/*.hip with the host side under ``-fsanitize=address`` (the device code as usual),
generates a C++ driver from
include/ivit.h that calls EVERY declared entry point with argument patterns that must be rejected by
validation or be no-ops (all-zero sizes and NULL pointers; all -1 sizes), sweeps the workspace
queries over the bench / test shapes, and drives the kernel-timing bookkeeping (ivit_ktime_*) with
real host buffers; then runs it. Exit status 0 and no AddressSanitizer report = pass.

    python tools/asan_abi.py [--out build_asan]      (tests/test_cpu_asan.py runs it)

Run on a CPU host only: with a GPU present the zero / negative patterns would still be no-ops or
validation errors, but nothing here needs one.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "visiontransformer-intention-prediction_amd")
HEADER = os.path.join(ROOT, "include", "ivit.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# host side instrumented (each -fsanitize= right after -Xarch_host); the device code is built as in the
# product (GPU ASan is not available) so the objects carry their real code objects
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-Xarch_host", "-fsanitize=address",
         "-Xarch_host", "-fno-omit-frame-pointer", "-Wno-unused-function", "-Wno-unused-command-line-argument"]


def prototypes():
    """[(ret, name, [(type, argname)])] of every ivit_* prototype."""
    txt = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    txt = re.sub(r"//[^\n]*", " ", txt)
    out = []
    for m in re.finditer(r"(const\s+char\s*\*|int|long)\s+(ivit_\w+)\s*\(([^)]*)\)\s*;", txt, flags=re.S):
        args = []
        a = " ".join(m.group(3).split())
        if a and a != "void":
            for part in a.split(","):
                part = part.strip()
                if "*" in part:
                    args.append(("ptr", part))
                else:
                    t = part.rsplit(" ", 1)[0].replace("const ", "").strip()
                    args.append((t, part))
        out.append((m.group(1), m.group(2), args))
    return out


def _val(t, pattern):
    if t == "ptr":
        return "nullptr"
    if t == "float":
        return "0.0f" if pattern == "zero" else "-1.0f"
    if t == "double":
        return "0.0" if pattern == "zero" else "-1.0"
    return "0" if pattern == "zero" else "-1"


def driver_source():
    # every call runs in a forked child, so one report names every entry point that fails (ASan
    # aborts the process at its first error)
    lines = ['#include <cstdio>', '#include <cstring>', '#include <sys/wait.h>', '#include <unistd.h>',
             '#include "ivit.h"', "",
             "static int failures = 0;",
             "template <class F> static void guarded(const char* what, F f) {",
             "  std::fflush(stdout);",
             "  const pid_t pid = fork();",
             "  if (pid == 0) { f(); std::fflush(stdout); _exit(0); }",
             "  int st = 0;",
             "  waitpid(pid, &st, 0);",
             "  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) { ++failures; std::printf(\"FAILED %s\\n\", what); }",
             "}", "",
             "int main() {",
             "  long calls = 0;", '  std::printf("%s\\n", ivit_version());']
    protos = prototypes()
    for ret, name, args in protos:
        if name in ("ivit_version", "ivit_last_error", "ivit_ktime_arm", "ivit_ktime_read"):
            continue
        for pattern in ("zero", "neg"):
            call = f"{name}({', '.join(_val(t, pattern) for t, _ in args)})"
            if ret == "int":
                body = f"(void){call}; (void)std::strlen(ivit_last_error());"
            else:
                body = f"volatile long v = {call}; (void)v;"
            lines.append(f'  guarded("{name} [{pattern}]", [] {{ {body} }}); ++calls;')
    # workspace queries over the shapes the product uses (bench B = 8 / 32, N = 4501 / 18001, ...)
    for ret, name, args in protos:
        if not name.endswith("_workspace") or ret != "long":
            continue
        for size in (1, 7, 64, 4501, 18001, 36008):
            vals = []
            for t, a in args:
                if t == "ptr":
                    vals.append("nullptr")
                elif t in ("int",):
                    vals.append("1")
                else:
                    vals.append(str(size))
            lines.append(f'  guarded("{name} [size {size}]", [] {{ volatile long v = {name}({", ".join(vals)}); '
                         f'(void)v; }}); ++calls;')
    # kernel-timing bookkeeping with real host buffers (nothing recorded without launches)
    lines += ["  {",
              "    double s[4], e[4]; long n = -1;",
              "    ivit_ktime_arm(1);",
              "    for (int tag = 0; tag < 3; ++tag) { if (ivit_ktime_read(tag, s, e, 4, &n) != 0 || n != 0) return 2; }",
              "    if (ivit_ktime_read(99, s, e, 4, &n) >= 0) return 3;  // unknown tag rejected",
              "    if (ivit_ktime_read(0, nullptr, nullptr, 4, &n) >= 0) return 4;  // null outputs rejected",
              "    if (ivit_ktime_read(0, nullptr, nullptr, 0, &n) != 0) return 5;  // count only",
              "    ivit_ktime_arm(0);",
              "    calls += 6;",
              "  }",
              '  std::printf("asan abi driver: %ld calls, %d failed\\n", calls, failures);',
              "  return failures ? 1 : 0;", "}"]
    return "\n".join(lines) + "\n", len(protos)


def build(out):
    os.makedirs(out, exist_ok=True)
    srcs = sorted(f for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".hip"))
    objs = []
    procs = []
    for f in srcs:
        o = os.path.join(out, f.replace(".hip", ".o"))
        src = os.path.join(PKG, "csrc", f)
        objs.append(o)
        if os.path.exists(o) and os.path.getmtime(o) >= max(
                [os.path.getmtime(src), os.path.getmtime(HEADER)] +
                [os.path.getmtime(os.path.join(PKG, "csrc", h)) for h in os.listdir(os.path.join(PKG, "csrc"))
                 if h.endswith(".h")]):
            continue
        procs.append(subprocess.Popen([HIPCC] + FLAGS + ["-c", src, "-o", o]))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("asan_abi: host-only compile failed")
    src, n = driver_source()
    drv = os.path.join(out, "abi_driver.cpp")
    with open(drv, "w") as fh:
        fh.write(src)
    exe = os.path.join(out, "abi_asan")
    # the driver is plain C++ (no HIP language mode); link with the ROCm clang and the HIP runtime
    cxx = os.path.join(os.path.dirname(os.path.realpath(HIPCC)), "..", "lib", "llvm", "bin", "clang++")
    if not os.path.exists(cxx):
        cxx = "/opt/rocm/lib/llvm/bin/clang++"
    asan = ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"]
    subprocess.run([cxx] + asan + ["-std=c++17", "-I", os.path.join(ROOT, "include"), "-c", drv, "-o", drv + ".o"],
                   check=True)
    subprocess.run([cxx] + asan + [drv + ".o"] + objs + ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib",
                                                         "-o", exe], check=True)
    return exe, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(PKG, "build_asan"))
    a = ap.parse_args()
    exe, n = build(a.out)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, env=env)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    if r.returncode != 0 or "ERROR: AddressSanitizer" in r.stderr:
        raise SystemExit(f"asan_abi: driver failed (status {r.returncode})")
    print(f"asan_abi: {n} entry points exercised, no AddressSanitizer report")


if __name__ == "__main__":
    main()
