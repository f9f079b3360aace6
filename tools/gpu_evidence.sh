set -u
# Round evidence: every -m gpu test, smoke, the default bench line (CPU baseline included),
# the DDP leg (--force-collectives), config 4 (eval B=32) and config 5 (800x1440).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-evidence}
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-collectives > gpurun_out/${TAG}_bench_force_collectives.json 2>gpurun_out/${TAG}_fc.err
rc=$?; echo "fc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_force_collectives.json')); print(d['collectives_world1'])"
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_eval_config4.json 2>gpurun_out/${TAG}_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --grid 800x1440 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_large_config5.json 2>gpurun_out/${TAG}_large.err
rc=$?; echo "large rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; [print(f, json.load(open('gpurun_out/${TAG}_'+f+'.json'))['value']) for f in ('bench_eval_config4','bench_large_config5')]"
