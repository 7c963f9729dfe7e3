set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python tools/batch_ab.py > $OUT/batch_ab.log 2>&1
echo rc=$?
