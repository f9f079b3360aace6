set -u
# attention: parity tests, micro-bench, and the FETCH_SIZE / WRITE_SIZE passes over tools/attn_once.py
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "attention" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ta_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ta_$TAG.log; [ $rc -eq 0 ] || exit $rc
TORCH_SDPA=0 timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/attn_$TAG.log; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${C}_$TAG -o run -- python3 tools/attn_once.py > gpurun_out/pmc_${C}_$TAG.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE_$TAG gpurun_out/pmc_WRITE_SIZE_$TAG > gpurun_out/attn_hbm_$TAG.json
