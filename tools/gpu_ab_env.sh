set -u
# Same-call A/B of an environment switch: op tests (pytest -k FILTER) with the default, the stamp
# anatomy and tools/block_bench.py for each value.   gpu_ab_env.sh VAR "v1 v0" FILTER TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; FILTER=$3; TAG=$4
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -k "$FILTER" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python tools/panel_stamps.py > gpurun_out/stamps_${TAG}_$v.txt 2>&1; rc=$?
  echo "$VAR=$v"; cut -c1-330 gpurun_out/stamps_${TAG}_$v.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
  env $VAR=$v BLAS_REF=0 timeout -k 10 200 python tools/block_bench.py > gpurun_out/bb_${TAG}_$v.txt 2>&1; rc=$?
  grep -vE "amdgpu.ids|wgrad" gpurun_out/bb_${TAG}_$v.txt; [ $rc -eq 0 ] || exit $rc
done
