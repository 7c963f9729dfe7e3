set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_stats.so timeout -k 10 300 python tools/bvh_stats.py --scenes ${SC:-cornell,scene0} --out $OUT/stats_${TAG:-s}.json > $OUT/stats_${TAG:-s}.log 2>&1
echo "rc=$?"
