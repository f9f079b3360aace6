set -u
# attention micro-bench + kernel stats + SQ anatomy (one GPU call). Usage: gpu_attn.sh TAG
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-attn}
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/attn_$TAG.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attnprof_$TAG -o run --output-format csv -- python3 tools/attn_once.py > gpurun_out/attnprof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_sq.sh $TAG tools/attn_once.py && python tools/pmc_anatomy.py gpurun_out/pmc_${TAG}_1 gpurun_out/pmc_${TAG}_2
