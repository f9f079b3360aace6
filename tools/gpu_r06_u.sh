cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
CNN_STEPS=10 timeout -k 10 400 python tools/cnn_bench.py > gpurun_out/r06_u_cnn_bench.json 2> gpurun_out/r06_u_cnn_bench.err
rc=$?; echo "cnn rc=$rc"; cat gpurun_out/r06_u_cnn_bench.json; tail -3 gpurun_out/r06_u_cnn_bench.err; exit $rc
