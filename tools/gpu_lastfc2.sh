set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_model.py tests/test_cnn.py tests/test_gpu_ops.py -k "not ops or bn or conv or cnn" -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_lf.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_lf.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_lf.json 2> gpurun_out/bench_lf.err
rc=$?; python -c "import json; d=json.load(open('gpurun_out/bench_lf.json')); print(d['ms_per_step'], d['value'])"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_quick.sh lf
