set -u
# LayerNorm / wide-kernel epilogue prefetch depth: isolated, then in the bench step (alternating).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in lnbase lncur; do echo "== $n"; IVIT_LIB=ab/lib_$n.so timeout -k 10 120 python tools/resid_ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
for rep in 1 2 3; do for n in lnbase lncur lnw4; do
  IVIT_LIB=ab/lib_$n.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab2_$n.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab2_$n.json')); print('$n', d['ms_per_step'])"
done; done
