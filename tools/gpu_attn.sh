set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -m gpu -p no:cacheprovider -k "attention" > gpurun_out/attn_tests.log 2>&1; rc=$?; echo "attn tests rc=$rc"; tail -2 gpurun_out/attn_tests.log
if [ $rc -le 1 ]; then timeout -k 10 300 python tools/attn_bench.py ${VARIANTS:-1 2 3 4} > gpurun_out/attn_bench.log 2>&1; echo "attn bench rc=$?"; cat gpurun_out/attn_bench.log; fi
