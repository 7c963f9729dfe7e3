# A/B timing + tests + per-variant HBM counters, one GPU call.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${TAG:-i}
pmc() {  # $1 name  $2 lib path
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmcab_fetch_$1_$T -o run --output-format csv \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmcab_$1_$T.log 2>&1 &&
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmcab_write_$1_$T -o run --output-format csv \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline >> $OUT/pmcab_$1_$T.log 2>&1
}
timeout -k 10 400 python tools/variant_bench.py ${VARIANTS:-wi wi4 flat} > $OUT/variants_$T.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu_$T.log 2>&1
echo "rc_tests=$?" > $OUT/ab_$T.status
pmc default "" && IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_wi4.so pmc wi4 &&
timeout -k 10 300 python bench.py > $OUT/bench_$T.json 2> $OUT/bench_$T.err
echo "rc_all=$?" >> $OUT/ab_$T.status
