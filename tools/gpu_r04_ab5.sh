set -u
# Patch weight-gradient reduce (16-B form): its tests, the isolated launch and the step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "patch" --timeout 120 --timeout-method thread > gpurun_out/ab5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/patch_bench.py wgrad 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab5 -o run --output-format csv -- python3 tools/patch_once.py wgrad > gpurun_out/prof_ab5.log 2>&1 || exit 1
grep -h "patch_wgrad" gpurun_out/prof_ab5/run_kernel_stats.csv | cut -c1-200
for rep in 1 2; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab5.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab5.json')); print('step', d['ms_per_step'])"; done
