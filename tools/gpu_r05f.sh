set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r05_f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_entry.py tests/test_gpu_model.py -x -q -k "nms or postprocess or config4" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/${T}_bench_eval.json 2>gpurun_out/${T}_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_eval.json')); print('eval', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profeval -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/${T}_profeval.log 2>&1
rc=$?; echo "prof eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r05_f_profeval/run_kernel_stats.csv')):
    if 'nms' in r['Name'] or 'trampoline' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, 'us')
PY
