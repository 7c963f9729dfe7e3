# GPU tests, then a variant A/B over all four scenes
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-vt2}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$T.log 2>&1 &&
IPT_VB_SPHERE=1 IPT_VB_NORTHSTAR=1 timeout -k 10 500 python tools/variant_bench.py ${VARIANTS:-base} > $OUT/variants_$T.log 2>&1
echo "rc=$?"
