set -u
# Same-call A/B of an attention environment switch: attention op tests with the first value, then
# tools/attn_bench.py alternating.   gpu_attn_ab.sh VAR "v1 v0 v1 v0"
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; first=${VALS%% *}
env $VAR=$first timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attention" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_attnab.log 2>&1
rc=$?; echo "tests ($VAR=$first): $(tail -1 gpurun_out/t_attnab.log)"; [ $rc -eq 0 ] || exit $rc
i=0
for v in $VALS; do
  i=$((i+1))
  env $VAR=$v TORCH_SDPA=0 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attnab_$i.txt 2>&1; rc=$?
  echo "$VAR=$v: $(grep -E '^fwd q2|^bwd q2' gpurun_out/attnab_$i.txt | cut -c1-40 | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
