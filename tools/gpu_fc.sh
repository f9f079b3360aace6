set -u
# DDP leg on one GPU: bench.py --force-collectives at several bucket sizes (plain step vs the
# world-1 RCCL bucketed step, same process), then the gloo / RCCL DDP tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fc}
for mb in 64 16 256; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-collectives --bucket-mb $mb > gpurun_out/fc_${TAG}_$mb.json 2> gpurun_out/fc_${TAG}_$mb.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/fc_${TAG}_$mb.json')); c=d['collectives_world1']; print('bucket_mb', $mb, 'plain', c['ms_per_step_plain'], 'buckets', c['ms_per_step_buckets'], 'overhead', c['overhead_ms'], 'n', c['buckets'])" || exit 1
done
