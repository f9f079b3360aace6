set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cnn.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests.log 2>&1; rc=$?; echo "cnn tests rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/cnn_tests.log | head -30; tail -3 gpurun_out/cnn_tests.log
exit $rc
