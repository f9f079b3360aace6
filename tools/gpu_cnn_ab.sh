set -u
# CNN variant: parity tests, then the train-step bench with the conv panel kernels on / off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_cnn.sh || exit $?
for v in 1 0; do
  IVIT_CONV_PANEL=$v timeout -k 10 300 python tools/cnn_bench.py > gpurun_out/cnn_bench_$v.json 2> gpurun_out/cnn_bench_$v.err
  rc=$?; echo "IVIT_CONV_PANEL=$v rc=$rc"; tail -c 600 gpurun_out/cnn_bench_$v.json
  [ $rc -eq 0 ] || exit $rc
done
