set -u
# Round evidence on the current tree: every -m gpu test, smoke, the default bench line with its
# attention intervals (roofline.frac recomputable: tools/kunion.py on the CSV), the rocprofv3
# kernel trace + stats of the profiled bench and the union JSON of the attention backward pair from
# it (bench.py reads it into roofline.frac_rocprof), config 4 (eval B = 32) and config 5 (800x1440).
#   bash tools/gpu_round.sh TAG [skip-tests]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-round}
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.txt; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --intervals-out gpurun_out/${TAG}_attn_intervals.csv > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; print(d['ms_per_step'], d['value'], r['frac'], r.get('frac_rocprof'), d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/kunion.py gpurun_out/${TAG}_prof/run_kernel_trace.csv attn_bwd_dq attn_bwd_dkv --flops 4.979e11 --json gpurun_out/${TAG}_attn_bwd_union.json
python tools/kunion.py gpurun_out/${TAG}_attn_intervals.csv attn_bwd_dq attn_bwd_dkv --flops 4.979e11 --json gpurun_out/${TAG}_attn_bwd_intervals_union.json
# HBM bytes per kernel: one FETCH_SIZE and one WRITE_SIZE pass (separate runs), summarised with the
# gfx950 corrections (tools/pmc_summary.py); bench.py reads the newest profiles/*_pmc_hbm.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmcf -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/${TAG}_pmcf.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmcw -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/${TAG}_pmcw.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmcf gpurun_out/${TAG}_pmcw "patch_wgrad|attn_bwd" > gpurun_out/${TAG}_pmc_hbm.json
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_eval_config4.json 2>gpurun_out/${TAG}_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --grid 800x1440 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_large_config5.json 2>gpurun_out/${TAG}_large.err
rc=$?; echo "large rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; [print(f, json.load(open('gpurun_out/${TAG}_'+f+'.json'))['value']) for f in ('bench_eval_config4','bench_large_config5')]"
