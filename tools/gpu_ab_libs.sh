set -u
# Same-call A/B of prebuilt libraries (tools/ab_build.sh): runs PROG with IVIT_LIB=ab/lib_<name>.so
# for each name, twice, alternating.  Usage: gpu_ab_libs.sh "<prog args>" name1 name2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PROG=$1; shift
for rep in 1 2; do
  for n in "$@"; do
    echo "== $n ($rep)"
    IVIT_LIB=ab/lib_$n.so TORCH_SDPA=0 timeout -k 10 300 python $PROG 2>&1 | grep -v "amdgpu.ids\|rel-L2" || exit 1
  done
done
