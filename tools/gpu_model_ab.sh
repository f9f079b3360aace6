set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_entry.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_gm.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_gm.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_ab.sh IVIT_CONV_PANEL "1 0 1 0"
