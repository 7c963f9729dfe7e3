set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python tools/tolerance_ab.py fastcast > $OUT/fastcast_tol.log 2>&1 &&
IPT_VB_ONLY=cornell,scene0 timeout -k 10 600 python tools/variant_bench.py qnodes fastcast > $OUT/fastcast_ab.log 2>&1
echo rc=$?
