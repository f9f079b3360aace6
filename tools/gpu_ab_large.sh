set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for E in "IVIT_GEMM_BIG=0" "IVIT_GEMM_BIG=1"; do
  env $E timeout -k 10 400 python bench.py --grid 800x1440 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abL_${E}_$rep.json 2>gpurun_out/abL_${E}_$rep.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/abL_${E}_$rep.json')); print('$E', d['ms_per_step'], 'ms', d['value'], 'samples/s')"
done; done
