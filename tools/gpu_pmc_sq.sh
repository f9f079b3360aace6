set -u
# SQ counter passes (issue / wait / MFMA-busy anatomy) over one program. Usage: gpu_pmc_sq.sh TAG prog.py
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; PROG=$2
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 $PROG > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc $TAG pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
