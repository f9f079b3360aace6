cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_model.py tests/test_gpu_entry.py tests/test_cnn.py > gpurun_out/r06_f_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_f_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_f_bench_eval_config4.json 2> gpurun_out/r06_f_eval.err
rc=$?; echo "eval rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/r06_f_bench_eval_config4.json')); print(d['ms_per_step'], d['value'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_f_evalprof -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r06_f_evalprof.log 2>&1
rc=$?; echo "evalprof rc=$rc"; grep -c "at::native" gpurun_out/r06_f_evalprof/run_kernel_stats.csv
