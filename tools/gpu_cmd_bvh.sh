# BVH round: GPU tests, per-scene A/B, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-bvh1}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu_$T.log 2>&1 &&
timeout -k 10 300 python tools/bench_scenes.py > $OUT/scenes_$T.jsonl 2> $OUT/scenes_$T.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$T.json 2> $OUT/bench_$T.err
echo "rc=$?"
