set -u
# AdamW chunked: its tests; then in-step A/B of the stream lead (LiDAR backward k blocks ahead).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_loss.py -x -q -k "adamw or guard" --timeout 120 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab3_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for k in 0 1 3; do
  IVIT_STREAM_LEAD=$k timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab3_l$k.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab3_l$k.json')); print('lead $k', d['ms_per_step'])"
done; done
