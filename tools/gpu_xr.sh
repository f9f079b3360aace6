set -u
# dK/dV row constants through the extra MFMA (IVIT_ATTN_XR=1, default) vs f32 row vectors (=0):
# attention tests through it, then timing, alternating.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "attention or attn" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_xr.log 2>&1
rc=$?; tail -3 gpurun_out/t_xr.log; [ $rc -eq 0 ] || exit $rc
for e in 1 0 1 0; do
  IVIT_ATTN_XR=$e TORCH_SDPA=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/ab_xr_$e.txt 2>&1; rc=$?
  echo "xr=$e: $(grep -E 'bwd q2|rel-L2' gpurun_out/ab_xr_$e.txt | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
