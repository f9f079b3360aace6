set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r05_g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "patch_wgrad_raster_exact or patch_embed" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_pw_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_pw_tests.txt; [ $rc -eq 0 ] || exit $rc
shift
bash tools/gpu_ab_libs.sh "tools/patch_bench.py wgrad" "$@" > gpurun_out/${T}_pw_ab.txt 2>&1; grep -v "patch matrix" gpurun_out/${T}_pw_ab.txt
