set -u
# Round 4 first GPU pass: every -m gpu test, then the default bench with the world-1 RCCL bucketed
# path timed beside the plain step (bench.py --force-collectives).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04a}
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-collectives > gpurun_out/bench_fc_$TAG.json 2> gpurun_out/bench_fc_$TAG.err
rc=$?; echo "bench fc rc=$rc"; tail -2 gpurun_out/bench_fc_$TAG.err
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/bench_fc_$TAG.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['collectives_world1'])"
