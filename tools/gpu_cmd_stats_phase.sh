# Work counters (IPT_BVH_STATS build) of all four bench scenes, then the
# per-phase cycle shares (IPT_PHASE_TIMING build) incl. the BVH scenes.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_AMD_LIB=inverse_path_tracer_amd/lib/variants/libipt_stats.so timeout -k 10 300 python tools/bvh_stats.py --out $OUT/bvh_stats.json > $OUT/bvh_stats.log 2>&1 &&
IPT_VB_NORTHSTAR=1 IPT_VB_SPHERE=1 timeout -k 10 300 python tools/phase_timing.py > $OUT/phase_${TAG:-ph}.log 2>&1
echo rc=$?
