set -u
# One GPU call: panel-conv parity tests, the conv microbench, and the small-ATen-kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-conv}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu -k "conv or bn or cnn" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/convbench_$TAG.txt 2>&1
rc=$?; echo "conv bench rc=$rc"; cat gpurun_out/convbench_$TAG.txt
[ $rc -eq 0 ] || exit $rc
true
rc=0
exit $rc
