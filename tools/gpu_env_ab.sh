set -u
# Same-call A/B of an environment switch on the headline step: gpu_env_ab.sh VAR "v1 v2" TAG [TESTFILTER]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; TAG=$3; FILT=${4:-}
if [ -n "$FILT" ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu -k "$FILT" -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_${TAG}_${v}_$rep.json 2>gpurun_out/b_${TAG}_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json')); print('$VAR=$v', d['ms_per_step'], 'ms', d['value'], 'sps', d['roofline']['per_step_ms'])"
  done
done
