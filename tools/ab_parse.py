"""Prints ms_per_step per library from a tools/gpu_ab_libs.sh log (gpurun_out/ab_cr.log or argv[1])."""
import sys
import json
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_cr.log"):
    if l.startswith("=="): print(l.strip(), end="  ")
    elif l.startswith("{"): print(json.loads(l)["ms_per_step"])
