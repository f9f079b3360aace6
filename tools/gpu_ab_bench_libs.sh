set -u
# Same-call A/B of prebuilt libraries on the full bench (tools/ab_build.sh): bench.py with
# IVIT_LIB=ab/lib_<name>.so for each name, twice, alternating.  Usage: gpu_ab_bench_libs.sh TAG name1 name2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for rep in 1 2; do
  for n in "$@"; do
    IVIT_LIB=ab/lib_$n.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${TAG}_${n}_$rep.json 2>gpurun_out/ab_${TAG}_${n}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${n}_$rep.json')); r=d['roofline']; print('$n', d['ms_per_step'], 'ms', d['value'], 'samples/s', 'attn_bwd', r['achieved'], r['frac'], 'iso', r['isolated']['ms'])"
  done
done
