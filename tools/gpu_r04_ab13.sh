set -u
# Wide kernels: two 256-thread workgroups per CU (default) vs one 512-thread workgroup per panel.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IVIT_WIDE_W=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "panel_wide or gelu_derivative" --timeout 120 --timeout-method thread > gpurun_out/ab13_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab13_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in 4 8; do
  IVIT_WIDE_W=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab13_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab13_$v.json')); print('wide_w $v', d['ms_per_step'])"
done; done
