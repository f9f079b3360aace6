set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests_$TAG.log
if [ $rc -le 1 ]; then timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_$TAG.json; fi
