set -u
# NMS exact division-free test (tests + eval + rocprof), SQ counters of the 32x32x16 and 16x16x32 attention
# forms side by side, the new default bench with its intervals and rocprof union
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r05_e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_entry.py tests/test_gpu_model.py -x -q -k "attention or nms or postprocess or config4" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/${T}_bench_eval.json 2>gpurun_out/${T}_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_eval.json')); print('eval', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profeval -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/${T}_profeval.log 2>&1
rc=$?; echo "prof eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
export ATTN_FORMS="000;111"
bash tools/gpu_pmc_sq.sh ${T}_attn tools/attn_once.py && python tools/pmc_anatomy.py gpurun_out/pmc_${T}_attn_1 gpurun_out/pmc_${T}_attn_2 > gpurun_out/${T}_attn_sq.txt
rc=$?; cat gpurun_out/${T}_attn_sq.txt; [ $rc -eq 0 ] || exit $rc
unset ATTN_FORMS
timeout -k 10 400 python bench.py --intervals-out gpurun_out/${T}_attn_intervals.csv > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_default.json')); r=d['roofline']; print(d['ms_per_step'], d['value'], r['frac'], r.get('isolated',{}).get('frac'), d['cpu_baseline']['value'], d['attn_mfma_util'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
