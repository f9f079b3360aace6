set -u
# Driver-shaped checks: smoke(), bench.py with no flags, and --gpus 2 on a one-GPU box (must fail loudly).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench default rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(d['ms_per_step'], d['value'], d['n_gpus'], d['cpu_baseline']['value'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
echo "bench --gpus 2 rc=$? (non-zero expected on one GPU)"; tail -2 gpurun_out/bench_g2.err
exit 0
