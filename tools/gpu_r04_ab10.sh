set -u
# Wide-kernel epilogue default changed to the LDS-tile form: the panel tests (both forms), the
# bf16 model tests, then the step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "panel or bf16" --timeout 200 --timeout-method thread > gpurun_out/ab10_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab10_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab10.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab10.json')); print('step', d['ms_per_step'])"; done
