set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_DEBUG_GRID=1 timeout -k 10 300 python tools/batch_ab.py > $OUT/batch_ab.log 2>&1 &&
IPT_SET_IL=1 timeout -k 10 300 python tools/batch_ab.py > $OUT/batch_ab_il.log 2>&1 &&
IPT_GRID_PER_CU=5 timeout -k 10 300 python tools/batch_ab.py > $OUT/batch_ab_g5.log 2>&1
echo rc=$?
