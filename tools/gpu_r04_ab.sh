set -u
# Round-4 A/B call: neck-fork DDP diagnostic, the touched kernels' GPU tests, patch weight-gradient
# bound diagnostics + forms, row-panel epilogue prefetch depth (isolated, then in the bench step).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IVIT_NECK_FORK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_ddp.log 2>&1
rc=$?; tail -3 gpurun_out/ab_ddp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "patch_wgrad_raster or resid_ln or dgrad_ln or panel" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for n in pbase pdiag1 pdiag2; do echo "== $n"; IVIT_LIB=ab/lib_$n.so timeout -k 10 120 python tools/patch_bench.py wgrad 2>&1 | grep -v amdgpu.ids || exit 1; done
for m in 1 2 0; do echo "== patch wgrad mode $m"; IVIT_PATCH_WGRAD_SPLIT=$m timeout -k 10 120 python tools/patch_bench.py wgrad 2>&1 | grep -v amdgpu.ids || exit 1; done
for n in lnbase ln3 ln5; do echo "== $n"; IVIT_LIB=ab/lib_$n.so timeout -k 10 120 python tools/resid_ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
for rep in 1 2; do for n in lnbase ln3 ln5; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$n.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', d['ms_per_step'])"
done; done
for m in 2 0; do
  IVIT_PATCH_WGRAD_SPLIT=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_p$m.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_p$m.json')); print('patch mode $m', d['ms_per_step'])"
done
for rep in 1 2; do for f in 0 1; do
  IVIT_NECK_FORK=$f timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_nf$f.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_nf$f.json')); print('neck fork $f', d['ms_per_step'])"
done; done
