set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ab.log 2>&1 &&
IPT_VB_SPHERE=1 IPT_VB_NORTHSTAR=1 timeout -k 10 600 python tools/variant_bench.py ${VARIANTS} > $OUT/ab.log 2>&1
echo rc=$?
