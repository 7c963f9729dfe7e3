set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu_s2.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench_s2.json 2> $OUT/bench_s2.err
echo "rc=$?"
