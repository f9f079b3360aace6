cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_entry.py -k "attention or kernel_exec or nms or post" > gpurun_out/r06_o_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_o_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_o_bench_eval_config4.json 2> gpurun_out/r06_o_eval.err
rc=$?; echo "eval rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/r06_o_bench_eval_config4.json')); print(d['ms_per_step'], d['value'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_o_evalprof -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r06_o_evalprof.log 2>&1
rc=$?; echo "evalprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh tools/attn_bench.py base dqskip > gpurun_out/r06_o_attn_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "==|kernels:|plain" gpurun_out/r06_o_attn_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_bench_libs.sh dqskip base dqskip
