set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bev_augment.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/aug_tests.log 2>&1; rc=$?; echo "aug tests rc=$rc"; tail -15 gpurun_out/aug_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python tools/augment_bench.py > gpurun_out/aug_bench.json 2> gpurun_out/aug_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/aug_bench.json; tail -3 gpurun_out/aug_bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aug -o aug -- python tools/augment_bench.py > gpurun_out/prof_aug.log 2>&1; rc=$?; echo "prof rc=$rc"
find gpurun_out/prof_aug -name "*stats*" | head
exit $rc
