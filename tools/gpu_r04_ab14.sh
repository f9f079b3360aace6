set -u
# Forward attention, four K/V stages (IVIT_ATTN_FWD_DEEP=1): attention tests with it, isolated
# timing both ways, then the step alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IVIT_ATTN_FWD_DEEP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/ab14_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab14_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do echo "== deep $v"; IVIT_ATTN_FWD_DEEP=$v timeout -k 10 200 python tools/attn_bench.py 2>&1 | grep -E "fwd q2|rel-L2" || exit 1; done
for rep in 1 2 3; do for v in 0 1; do
  IVIT_ATTN_FWD_DEEP=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab14_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab14_$v.json')); print('deep $v', d['ms_per_step'], d['roofline']['per_step_ms'])"
done; done
