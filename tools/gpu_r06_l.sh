cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in 4096 4224 4501 4608; do
  echo "== N=$n"
  TORCH_SDPA=0 timeout -k 10 200 python tools/attn_bench.py $n || exit $?
done > gpurun_out/r06_l_attn_tiles.txt 2>&1
rc=$?; grep -E "==|kernels" gpurun_out/r06_l_attn_tiles.txt; exit $rc
