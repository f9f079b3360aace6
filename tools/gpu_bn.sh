set -u
# BatchNorm partial sums, 8 columns per thread: BN / model / CNN parity tests, bench step and
# kernel trace (compare bn_partial8_kernel with bn_partial_kernel in profiles/r02_v6_*).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-bn}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "batchnorm or small or stride2 or regrid or cnn or full_grid or fusion" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/tests_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$TAG.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
