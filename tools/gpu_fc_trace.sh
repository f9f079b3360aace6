set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fct}
for f in 0 1; do
  FORCE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$f -o run --output-format csv -- python tools/fc_trace.py 5 > gpurun_out/fct_${TAG}_$f.log 2>&1 || exit 1
  grep 'ms/step' gpurun_out/fct_${TAG}_$f.log
done
