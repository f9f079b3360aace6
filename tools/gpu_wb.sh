set -u
# Grouped block wgrad: op tests, A/B benches (grouped vs per-GEMM wgrad; 256x128 / 256x256 conv
# tiles), kernel-trace stats of the default.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-wb}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "vit_block_wgrad or adamw or conv or patch" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$T.log 2>&1
rc=$?; tail -3 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
IVIT_GEMM_WM4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or linear" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t4_$T.log 2>&1
rc=$?; tail -3 gpurun_out/t4_$T.log; [ $rc -eq 0 ] || exit $rc
for cfg in "default" "IVIT_GROUP_WGRAD=0" "default" "IVIT_GROUP_WGRAD=0"; do
  if [ "$cfg" = default ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$T.json 2>gpurun_out/b_$T.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_$T.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_$T.json').read().strip().splitlines()[-1]);print('$cfg', d['ms_per_step'], d['value'], d['loss'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
