set -u
# Same-call A/B of an attention kernel switch: op tests with the candidate, isolated timing of each
# value, then the headline step.   gpu_attn_env.sh VAR "v0 v1 ..." TAG
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; TAG=$3
LAST=${VALS##* }
env $VAR=$LAST timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu -k "attention" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "tests($VAR=$LAST) rc=$rc"; tail -2 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in $VALS; do
  env $VAR=$v TORCH_SDPA=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/ab_${TAG}_$v.txt 2>&1; rc=$?
  echo "$VAR=$v"; grep -E 'fwd q2|bwd q2|rel-L2' gpurun_out/ab_${TAG}_$v.txt; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_${TAG}_${v}_$rep.json 2>gpurun_out/b_${TAG}_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json')); print('$VAR=$v', d['ms_per_step'], 'ms', d['value'], 'sps', d['roofline']['per_step_ms'])"
  done
done
