set -u
# dK/dV 16x16x32 as the default: in-step A/B against v3; NMS mask / scan rework (tests, eval bench, rocprof)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r05_c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_entry.py -x -q -k "attention or nms or postprocess or panel" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${T}_tests.txt; [ $rc -eq 0 ] || exit $rc
ATTN_VARIANTS="IVIT_ATTN_FWD16=0;IVIT_ATTN_FWD16=1" TORCH_SDPA=0 timeout -k 10 300 python tools/attn_bench.py > gpurun_out/${T}_attn_bench.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_attn_bench.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    IVIT_ATTN_FWD16=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_ab_fwd16_${v}_$rep.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('gpurun_out/${T}_ab_fwd16_${v}_$rep.json')); r=d['roofline']; print('FWD16=$v', d['ms_per_step'], d['value'], r['frac'], r.get('isolated',{}).get('frac'), r['per_step_ms'])"
  done
done
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/${T}_bench_eval.json 2>gpurun_out/${T}_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_eval.json')); print('eval', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profeval -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/${T}_profeval.log 2>&1
rc=$?; echo "prof eval rc=$rc"; exit $rc
