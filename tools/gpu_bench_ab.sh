set -u
# Same-call A/B of an environment switch on the headline bench: gpu_bench_ab.sh VAR "a b a b"
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; i=0
for v in $VALS; do
  i=$((i+1))
  env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bab_$i.json 2> gpurun_out/bab_$i.err
  rc=$?; echo "$VAR=$v: $(python -c "import json,sys; d=json.load(open('gpurun_out/bab_$i.json')); print(d['ms_per_step'], d['value'])" 2>&1)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bab_$i.err; exit $rc; }
done
