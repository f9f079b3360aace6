set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; VARS=${VARS:-5 8 9}
for v in $VARS; do
IVIT_ATTN_FWD_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/tests_attn_${TAG}_$v.log 2>&1
rc=$?; echo "attn tests v$v rc=$rc"; tail -2 gpurun_out/tests_attn_${TAG}_$v.log
[ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/attn_bench.py $VARS > gpurun_out/attn_$TAG.log 2>&1
rc=$?; echo "attn bench rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_$TAG.log
exit $rc
