set -u
# Kernel-trace stats of a short bench run (+ optional extra python diagnostic).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -c 600 gpurun_out/prof_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${2:-}" ]; then
  timeout -k 10 300 python3 $2 > gpurun_out/diag_$TAG.txt 2>&1
  rc=$?; echo "diag rc=$rc"; head -50 gpurun_out/diag_$TAG.txt
fi
exit $rc
