set -u
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/wgrad_bench.py --modes 1,2 > gpurun_out/wbench.txt 2>&1; rc=$?; tail -4 gpurun_out/wbench.txt; exit $rc
