set -u
# dK/dV v4 (IVIT_ATTN_DKV_V4=1): attention tests through it, then timing vs v3.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
IVIT_ATTN_DKV_V4=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attention" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_v4.log 2>&1
rc=$?; tail -3 gpurun_out/t_v4.log; [ $rc -eq 0 ] || exit $rc
for e in 0 1 2 0 1 2; do
  IVIT_ATTN_DKV_V4=$e TORCH_SDPA=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/ab_v4_$e.txt 2>&1; rc=$?
  echo "v4=$e: $(grep -E 'bwd q2|rel-L2' gpurun_out/ab_v4_$e.txt | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
