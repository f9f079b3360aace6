cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_ad_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_ad_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_ad_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r06_ad_smoke.txt; exit $rc
