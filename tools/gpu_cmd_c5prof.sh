set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run --output-format csv -- python3 $R/tools/bench_c5.py --steps 20 --warmup 3 --total 23 > $OUT/prof_c5.log 2>&1
echo rc=$?
