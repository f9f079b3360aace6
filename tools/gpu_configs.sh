set -u
# Config-5 / config-4 coverage: the large-grid parity tests, the eval (config 4) bench and a
# large-grid (config 5, 800x1440) single-GPU train bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "large_grid" > gpurun_out/tests_large_$TAG.log 2>&1
rc=$?; echo "large tests rc=$rc"; tail -5 gpurun_out/tests_large_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode eval --steps 5 --warmup 2 > gpurun_out/bench_eval_$TAG.json 2> gpurun_out/bench_eval_$TAG.err
rc=$?; echo "eval bench rc=$rc"; tail -c 1200 gpurun_out/bench_eval_$TAG.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --grid 800x1440 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bench_large_$TAG.json 2> gpurun_out/bench_large_$TAG.err
rc=$?; echo "large bench rc=$rc"; tail -c 1200 gpurun_out/bench_large_$TAG.json
exit $rc
