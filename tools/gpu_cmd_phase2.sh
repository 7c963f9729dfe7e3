set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-ph}
timeout -k 10 300 python tools/phase_timing.py > $OUT/phase_$T.log 2>&1 &&
timeout -k 10 400 python tools/variant_bench.py ${VARIANTS:-base} > $OUT/variants_$T.log 2>&1
echo "rc=$?"
