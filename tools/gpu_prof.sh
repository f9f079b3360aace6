set -u
# rocprofv3 kernel summary of a short default bench (the round's kernel-stats evidence).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/kstat_top.py gpurun_out/prof_$TAG/run_kernel_stats.csv 2>/dev/null | head -30
