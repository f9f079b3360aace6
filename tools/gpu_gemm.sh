set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "linear or conv or patch" > gpurun_out/tests_gemm_$TAG.log 2>&1
rc=$?; echo "op tests rc=$rc"; tail -3 gpurun_out/tests_gemm_$TAG.log
[ $rc -eq 0 ] || exit $rc
GEMM_VARIANTS=0,1 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_$TAG.log 2>&1
rc=$?; echo "gemm bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do IVIT_GEMM_PERSIST=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_p$v.json 2>gpurun_out/bench_${TAG}_p$v.err || exit 1; echo "p$v"; cut -c1-330 gpurun_out/bench_${TAG}_p$v.json; done
