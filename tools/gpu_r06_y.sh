cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_entry.py tests/test_gpu_model.py -k "nms or post or config4" > gpurun_out/r06_y_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_y_tests.txt; [ $rc -eq 0 ] || exit $rc
for n in base scan2; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_y_prof_$n -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r06_y_prof_$n.log 2>&1 || exit 1
  python3 - $n <<'PY'
import csv, sys
n = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/r06_y_prof_{n}/run_kernel_stats.csv")):
    if "nms" in r["Name"] or "post" in r["Name"]:
        print(n, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
for rep in 1 2; do
  for n in base scan2; do
    IVIT_LIB=ab/lib_$n.so timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_y_eval_${n}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06_y_eval_${n}_$rep.json')); print('$n', d['ms_per_step'], d['value'], d.get('kept_boxes_per_step'))"
  done
done
