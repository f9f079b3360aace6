set -u
# Engine GEMM knob in the step: IVIT_GEMM_BIG unset vs 1 (256-row tiles where they pay), alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do for v in 0 1; do
  IVIT_GEMM_BIG=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab11_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab11_$v.json')); print('gemm_big $v', d['ms_per_step'])"
done; done
