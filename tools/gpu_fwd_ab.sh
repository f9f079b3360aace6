set -u
# Attention forward without the spilling tail body: attention parity tests, the isolated kernel
# (tools/attn_bench.py), the bench step, a kernel trace and a FETCH/WRITE PMC pair.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fw}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention or timing or small or full_grid or regrid" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/tests_$TAG.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_$TAG.log 2>&1
rc=$?; echo "attn rc=$rc"; head -4 gpurun_out/attn_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$TAG.json) $(grep -o '"per_step_ms": {[^}]*}' gpurun_out/bench_$TAG.json)"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw_$TAG.log 2>&1
rc=$?; echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$TAG.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"
exit $rc
