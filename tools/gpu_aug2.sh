set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err; rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_plain.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --augment > gpurun_out/bench_aug.json 2> gpurun_out/bench_aug.err; rc=$?; echo "bench aug rc=$rc"; cut -c1-400 gpurun_out/bench_aug.json
exit $rc
