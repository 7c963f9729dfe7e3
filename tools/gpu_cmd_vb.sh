set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_VB_SPHERE=1 IPT_VB_NORTHSTAR=1 IPT_VB_ONLY=${VB_ONLY:-sphere,northstar,cornell} timeout -k 10 600 python tools/variant_bench.py ${VARIANTS} > $OUT/vb_${TAG:-x}.log 2>&1
echo rc=$?
