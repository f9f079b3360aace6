cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_ab_libs.sh tools/attn_bench.py base stg4 stg10 stg24 > gpurun_out/r06_e_attn_stagger.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "==|kernels:" gpurun_out/r06_e_attn_stagger.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for c in 1 0; do
  IVIT_CONCURRENT_STREAMS=$c timeout -k 10 300 python bench.py --mode eval --steps 10 --warmup 2 > gpurun_out/r06_e_eval_cs${c}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06_e_eval_cs${c}_$rep.json')); print('eval concurrent=$c', d['ms_per_step'], d['value'])"
done; done
