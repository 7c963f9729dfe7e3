# Per-phase cycle shares of the current kernels (IPT_PHASE_TIMING build) on
# the small scenes and the north-star BVH scene.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-ph3}
IPT_VB_NORTHSTAR=1 timeout -k 10 300 python tools/phase_timing.py > $OUT/phase_$T.log 2>&1
echo "rc=$?"
