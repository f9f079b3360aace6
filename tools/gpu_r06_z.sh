cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_entry.py tests/test_gpu_model.py -k "post or pipeline or config4 or eval" > gpurun_out/r06_z_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06_z_tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    IVIT_AB_POST_SERIAL=$v timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_z_eval_serial${v}_$rep.json 2> gpurun_out/r06_z_eval_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06_z_eval_serial${v}_$rep.json')); print('serial$v', d['ms_per_step'], d['value'], d.get('kept_boxes_per_step'))"
  done
done
