set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== fused"; timeout -k 10 300 python tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== old"; IVIT_ATTN_BWD_OLD=1 TORCH_SDPA=0 timeout -k 10 300 python tools/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
