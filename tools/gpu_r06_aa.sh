cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_ops.py -k "nms" > gpurun_out/r06_aa_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/r06_aa_tests.txt | tail -12; exit $rc
