set -u
# Differing patch grids: generic patch embedding, bilinear re-grid kernels, model vs golden.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rg}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "bilinear or patch16 or regrid or stride2" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/tests_$TAG.log | tail -30
exit $rc
