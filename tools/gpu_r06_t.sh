cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py tests/test_cnn.py tests/test_gpu_model.py -k "batchnorm or bn or cnn or fusion or conv" > gpurun_out/r06_t_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_t_tests.txt; exit $rc
