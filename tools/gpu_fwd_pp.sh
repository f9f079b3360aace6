set -u
# Ping-pong attention forward: op tests, isolated timing of IVIT_ATTN_FWD 0 / 1 / 2, then the step A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu -k "attention or adamw" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 2; do
  IVIT_ATTN_FWD=$v TORCH_SDPA=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/ab_${TAG}_$v.txt 2>&1; rc=$?
  echo "fwd=$v"; grep -E 'fwd|rel-L2' gpurun_out/ab_${TAG}_$v.txt; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in 0 1 2; do
    IVIT_ATTN_FWD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_${TAG}_${v}_$rep.json 2>gpurun_out/b_${TAG}_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json')); print('fwd=$v', d['ms_per_step'], 'ms', d['value'], 'sps', d['roofline']['per_step_ms'])"
  done
done
