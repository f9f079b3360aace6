cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r06_p_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > gpurun_out/r06_p_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; ls gpurun_out/r06_p_prof; exit $rc
