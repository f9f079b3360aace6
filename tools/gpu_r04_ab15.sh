set -u
# Stream interleave granularity (IVIT_STREAM_CHUNK: ViT steps per turn), alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do for v in 1 2 3; do
  IVIT_STREAM_CHUNK=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab15_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab15_$v.json')); print('chunk $v', d['ms_per_step'])"
done; done
