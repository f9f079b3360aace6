cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in scan2 anat; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_w_prof_$n -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r06_w_prof_$n.log 2>&1 || exit 1
  python3 - $n <<'PY'
import csv, sys
n = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/r06_w_prof_{n}/run_kernel_stats.csv")):
    if "nms_scan" in r["Name"]:
        print(n, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
