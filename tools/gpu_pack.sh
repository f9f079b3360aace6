set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -k "adamw or pack or full_grid" -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_pk.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests_pk.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_quick.sh pk
