set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_entry.py tests/test_cnn.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/entry_tests.log 2>&1; rc=$?; echo "entry tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/entry_tests.log | head -20; tail -3 gpurun_out/entry_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/cnn_bench.py > gpurun_out/cnn_bench.json 2> gpurun_out/cnn_bench.err; rc=$?; echo "cnn bench rc=$rc"; cat gpurun_out/cnn_bench.json; tail -3 gpurun_out/cnn_bench.err
[ $rc -eq 0 ] || exit $rc
CNN_STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o cnn -- python3 tools/cnn_bench.py > gpurun_out/prof_cnn.log 2>&1; rc=$?; echo "prof rc=$rc"
exit $rc
