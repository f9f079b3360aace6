set -u
# Fused patch-embed forward: mode A/B timings, then SQ anatomy and HBM / L2 counter passes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 120 python3 tools/patch_once.py 0 1 2 3 0 > gpurun_out/patch_modes_$TAG.log 2>&1; rc=$?; cat gpurun_out/patch_modes_$TAG.log; [ $rc -eq 0 ] || exit $rc
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
P3="FETCH_SIZE"
P4="TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_patch_${TAG}_$i -o run -- python3 tools/patch_once.py ${PO_ARGS:-} > gpurun_out/pmc_patch_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
