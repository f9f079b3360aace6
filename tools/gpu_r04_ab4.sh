set -u
# AdamW: chunked vs 2D-grid launch, isolated (tools/adamw_bench.py) and in the bench step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 0 1 0 1; do echo "== chunked=$c"; IVIT_ADAMW_CHUNKED=$c timeout -k 10 120 python tools/adamw_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
for rep in 1 2; do for c in 0 1; do
  IVIT_ADAMW_CHUNKED=$c timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab4_c$c.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab4_c$c.json')); print('chunked $c', d['ms_per_step'])"
done; done
