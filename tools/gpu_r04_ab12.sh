set -u
# Neck conv outputs in the compute dtype (IVIT_NECK_BF16): bf16 model parity tests, then in-step A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab12_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab12_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in 0 1; do
  IVIT_NECK_BF16=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab12_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab12_$v.json')); print('neck_bf16 $v', d['ms_per_step'], d['loss'])"
done; done
