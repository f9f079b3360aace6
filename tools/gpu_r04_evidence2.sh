set -u
# Round-4 evidence, part 2: rocprofv3 kernel summary of a short default bench, the HBM counter
# passes (FETCH_SIZE, WRITE_SIZE: one run each) over the same command with the patch weight
# gradient listed per launch (LiDAR / map split), and the attention SQ anatomy.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04_x}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/kstat_top.py gpurun_out/prof_$TAG/run_kernel_stats.csv 2>/dev/null | head -24
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$TAG.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw_$TAG.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG patch_wgrad > gpurun_out/${TAG}_pmc_hbm.json
rc=$?; echo "summary rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_attn.sh $TAG > gpurun_out/${TAG}_attn.txt 2>&1
rc=$?; echo "attn rc=$rc"; tail -30 gpurun_out/${TAG}_attn.txt; exit $rc
