set -u
# A/B of env-selected variants on the full bench (same box, back to back). Usage: gpu_ab.sh TAG "ENV1" "ENV2" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for rep in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${TAG}_${i}_$rep.json 2>gpurun_out/ab_${TAG}_${i}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${i}_$rep.json')); print('$E', d['ms_per_step'], 'ms', d['value'], 'samples/s', 'attn', d['roofline']['achieved'])"
  done
done
