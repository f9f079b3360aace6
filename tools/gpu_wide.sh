set -u
# Wide row-panel kernels: op tests, stamp anatomy, block bench (EV=1 default) and the EV=0 A/B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "panel" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_wide.log 2>&1
rc=$?; tail -3 gpurun_out/t_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/panel_stamps.py > gpurun_out/stamps_wide.txt 2>&1; rc=$?; cat gpurun_out/stamps_wide.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for e in 1 0; do
  IVIT_WIDE_EPI=$e BLAS_REF=0 timeout -k 10 200 python tools/block_bench.py > gpurun_out/bb_wide_$e.txt 2>&1; rc=$?
  echo "epi=$e"; grep -E "qkv \(panel|fc1 \+ GELU|fc2 dgrad x|proj dgrad" gpurun_out/bb_wide_$e.txt; [ $rc -eq 0 ] || exit $rc
done
