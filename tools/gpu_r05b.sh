set -u
# attention dK/dV 16x16x32 A/B (tests + isolated kernel times) and the NMS rewrite (bit-exact tests + eval bench)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_entry.py -x -q -k "attention or nms or config4 or postprocess or panel" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r05_b_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_b_tests.txt; [ $rc -eq 0 ] || exit $rc
ATTN_VARIANTS="IVIT_ATTN_DKV16=0;IVIT_ATTN_DKV16=1" TORCH_SDPA=0 timeout -k 10 300 python tools/attn_bench.py > gpurun_out/r05_b_attn_bench.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05_b_attn_bench.txt; [ $rc -eq 0 ] || exit $rc
WIDE_AB="IVIT_WIDE_PERSIST=0;IVIT_WIDE_PERSIST=1;IVIT_WIDE_PERSIST=2;IVIT_WIDE_PERSIST=3;IVIT_WIDE_PERSIST=5" BLAS_REF=0 timeout -k 10 300 python tools/block_bench.py > gpurun_out/r05_b_wide_ab.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05_b_wide_ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r05_b_bench_eval.json 2>gpurun_out/r05_b_eval.err
rc=$?; echo "eval rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/r05_b_bench_eval.json')); print('eval', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b_profeval -o run --output-format csv -- python3 bench.py --mode eval --steps 3 --warmup 1 > gpurun_out/r05_b_profeval.log 2>&1
rc=$?; echo "prof eval rc=$rc"; exit $rc
