cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py tests/test_gpu_model.py -k "attention or full_grid_bf16" > gpurun_out/r06_ac_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_ac_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_libs.sh tools/attn_bench.py base bns3 bns4 > gpurun_out/r06_ac_attn_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "==|kernels:" gpurun_out/r06_ac_attn_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_bench_libs.sh bns base bns4
