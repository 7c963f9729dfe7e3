# Round bench + profiles: bench.py (with CPU baseline), rocprof kernel-trace stats,
# FETCH/WRITE PMC passes, C5 loop, per-scene A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-full}
timeout -k 10 400 python bench.py > $OUT/bench_$T.json 2> $OUT/bench_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/prof_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_write_$T.log 2>&1 &&
timeout -k 10 300 python tools/bench_c5.py > $OUT/c5_$T.json 2> $OUT/c5_$T.err &&
timeout -k 10 300 python tools/bench_scenes.py > $OUT/scenes_$T.jsonl 2> $OUT/scenes_$T.err
echo "rc=$?"
