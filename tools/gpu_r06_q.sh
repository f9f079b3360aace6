cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_cnn.py -k "conv or bn or batchnorm or fusion or full_grid or head" > gpurun_out/r06_q_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_q_tests.txt; [ $rc -eq 0 ] || exit $rc
for n in base ring; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_q_prof_$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-isolated --no-cpu-baseline > gpurun_out/r06_q_prof_$n.log 2>&1 || exit 1
  python3 - $n <<'PY'
import csv, sys
n = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r06_q_prof_{n}/run_kernel_stats.csv")))
for r in rows:
    if "conv" in r["Name"]:
        print(n, r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
bash tools/gpu_ab_bench_libs.sh ring base ring
