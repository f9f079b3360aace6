set -u
# Forward stream stagger A/B (IVIT_STREAM_STAGGER), three alternating pairs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do for v in 0 1; do
  IVIT_STREAM_STAGGER=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab6_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab6_$v.json')); print('stagger $v', d['ms_per_step'], d['loss'])"
done; done
