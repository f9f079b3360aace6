cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_pmc_sq.sh r06_ab_final tools/attn_once.py || exit 1
python tools/pmc_anatomy.py gpurun_out/pmc_r06_ab_final_1 gpurun_out/pmc_r06_ab_final_2 > gpurun_out/r06_ab_attn_sq_final.txt
cat gpurun_out/r06_ab_attn_sq_final.txt
