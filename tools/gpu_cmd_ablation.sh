set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
IPT_VB_SPHERE=1 timeout -k 10 400 python tools/variant_bench.py notrav > $OUT/variants_nt.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_nt.json 2> $OUT/bench_nt.err
echo "rc=$?"
