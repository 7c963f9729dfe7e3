# Round measurement: the driver's default bench line, then the rocprofv3
# kernel-trace summary and the FETCH_SIZE / WRITE_SIZE passes of the C2
# command (no secondary workloads), each GPU step under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-meas}
timeout -k 10 400 python bench.py > $OUT/bench_full_$T.json 2> $OUT/bench_full_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/prof_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_fetch_$T.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write_$T -o run --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmc_write_$T.log 2>&1
echo "rc=$?"
