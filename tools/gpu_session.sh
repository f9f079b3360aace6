set -u
# One GPU call: model / CNN / conv / BN tests, the headline bench + kernel stats, then the config 4 / 5
# benches (tools/gpu_configs.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-s}
bash tools/gpu_lastfc2.sh || exit $?
bash tools/gpu_configs.sh $TAG
