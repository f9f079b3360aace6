set -u
# Kernel-execution timing hook: its GPU test, the q2 attention tests, a bench line and the
# kernel-trace stats of the same bench command (the roofline ms must agree with rocprof's).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-kt}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "timing or q2" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 1800 gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -c 600 gpurun_out/prof_$TAG.log
exit $rc
