cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_entry.py tests/test_gpu_ops.py -k "postprocess or nms or attention or kernel_exec" > gpurun_out/r06_a_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_a_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_model.py -k config4_eval > gpurun_out/r06_a_tests_c4.txt 2>&1
rc=$?; echo "c4 rc=$rc"; tail -3 gpurun_out/r06_a_tests_c4.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_a_bench_eval_config4.json 2> gpurun_out/r06_a_eval.err
rc=$?; echo "eval rc=$rc"; cat gpurun_out/r06_a_bench_eval_config4.json | head -c 600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_a_evalprof -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r06_a_evalprof.log 2>&1
rc=$?; echo "evalprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/r06_a_attn_bench.txt 2>&1
rc=$?; echo "attn_bench rc=$rc"; cat gpurun_out/r06_a_attn_bench.txt | head -20
