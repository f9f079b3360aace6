set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; BV=${BV:-3}
IVIT_ATTN_DKV_VARIANT=$BV timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/tests_attnb_${TAG}.log 2>&1
rc=$?; echo "attn tests dkv v$BV rc=$rc"; tail -2 gpurun_out/tests_attnb_${TAG}.log
[ $rc -eq 0 ] || exit $rc
BWD_VARIANTS=${BWDS:-2,3} timeout -k 10 300 python tools/attn_bench.py 10 > gpurun_out/attnb_$TAG.log 2>&1
rc=$?; echo "attn bench rc=$rc"; grep -v amdgpu.ids gpurun_out/attnb_$TAG.log
exit $rc
