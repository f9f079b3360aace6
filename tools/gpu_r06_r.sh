cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_model.py tests/test_gpu_ddp.py tests/test_gpu_entry.py > gpurun_out/r06_r_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_r_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_r_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r06_r_smoke.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    IVIT_AB_NECK_FORK=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06_r_fork${v}_$rep.json 2>gpurun_out/r06_r_fork${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06_r_fork${v}_$rep.json')); print('fork$v', d['ms_per_step'], d['value'])"
  done
done
