set -u
# Round-5 first call: every -m gpu test, the default bench with its attention intervals, the rocprofv3
# kernel trace of the profiled bench (union JSON for frac_rocprof), the --force-collectives trace
# (which queues the RCCL kernels use), config 4 (eval) kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05_a}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --intervals-out gpurun_out/${TAG}_attn_intervals.csv > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; print(d['ms_per_step'], d['value'], r['frac'], r.get('isolated',{}).get('frac'), d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_proffc -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --force-collectives > gpurun_out/${TAG}_proffc.log 2>&1
rc=$?; echo "prof fc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_profeval -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/${TAG}_profeval.log 2>&1
rc=$?; echo "prof eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-collectives > gpurun_out/${TAG}_bench_force_collectives.json 2>gpurun_out/${TAG}_fc.err
rc=$?; echo "fc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_force_collectives.json')); print(d['collectives_world1'])"
