set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_AMD_LIB=inverse_path_tracer_amd/lib/variants/libipt_stats.so timeout -k 10 300 python tools/bvh_stats.py --scenes northstar,sphere > $OUT/bvh_stats.log 2>&1 && cp profiles/bvh_stats.json $OUT/ &&
IPT_VB_ONLY=northstar,sphere,scene0 IPT_VB_NORTHSTAR=1 IPT_VB_SPHERE=1 timeout -k 10 300 python tools/phase_timing.py > $OUT/phase_northstar.log 2>&1
echo rc=$?
