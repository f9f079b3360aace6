set -u
# Wide-kernel epilogue form in the step: IVIT_WIDE_EPI=1 (default: transposed for QS / GELUD, LDS tile
# for GELU / DGELU / DMUL) vs 0 (LDS tile for all), alternating.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3 4; do for v in 1 0; do
  IVIT_WIDE_EPI=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab9_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab9_$v.json')); print('wide_epi $v', d['ms_per_step'])"
done; done
