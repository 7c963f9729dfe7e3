set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "adjoint or bvh or large" > $OUT/pytest_gpu_$T.log 2>&1 &&
timeout -k 10 300 python tools/bench_scenes.py --scenes sphere,clutter > $OUT/scenes_$T.jsonl 2> $OUT/scenes_$T.err &&
IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_stats.so timeout -k 10 200 python tools/bvh_stats.py > $OUT/bvhstats_$T.json 2>&1
echo "rc=$?"
