set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 900 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -le 1 ]; then timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-900; fi
if [ $rc -le 1 ]; then timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1; echo "prof rc=$?"; fi
