set -u
# BatchNorm passes: rows per partial block / rows per load batch. Tests, isolated (tools/cnn_bench-like
# neck timing via the bench), in-step A/B alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "bn or batchnorm or conv" --timeout 120 --timeout-method thread > gpurun_out/ab8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab8_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for n in bnbase bn32b4 bn32b2 bn64b2; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab8_$n.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab8_$n.json')); print('$n', d['ms_per_step'])"
done; done
IVIT_LIB=ab/lib_bnbase.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab8a -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab8b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
grep -h "bn_" gpurun_out/prof_ab8a/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
echo ---
grep -h "bn_" gpurun_out/prof_ab8b/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
