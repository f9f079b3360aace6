cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_model.py -k config1 > gpurun_out/r06_d_config1.txt 2>&1
rc=$?; echo "config1 rc=$rc"; tail -30 gpurun_out/r06_d_config1.txt
