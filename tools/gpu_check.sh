set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_ops.py -q -m gpu -p no:cacheprovider > gpurun_out/ops.log 2>&1; rc=$?; echo "ops rc=$rc"
if [ $rc -le 1 ]; then timeout -k 10 900 python -m pytest tests/test_gpu_model.py -q -m gpu -p no:cacheprovider > gpurun_out/model.log 2>&1; rc=$?; echo "model rc=$rc"; fi
if [ $rc -le 1 ]; then timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; fi
tail -5 gpurun_out/ops.log; tail -5 gpurun_out/model.log 2>/dev/null; tail -3 gpurun_out/bench.log 2>/dev/null
