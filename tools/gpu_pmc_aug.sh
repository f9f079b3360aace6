set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
AUG_B=8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_aug -o aug --output-format csv -- python3 tools/augment_bench.py > gpurun_out/pmcf_aug.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
AUG_B=8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_aug -o aug --output-format csv -- python3 tools/augment_bench.py > gpurun_out/pmcw_aug.log 2>&1; rc=$?; echo "pmc write rc=$rc"
exit $rc
