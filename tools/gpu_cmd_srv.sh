set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd $R
T=${TAG:-srv}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bvh or large or sphere" > $OUT/pytest_gpu_$T.log 2>&1 &&
IPT_VB_SPHERE=1 timeout -k 10 400 python tools/variant_bench.py ${VARIANTS:-srv5 nosrv} > $OUT/variants_$T.log 2>&1 &&
timeout -k 10 300 python tools/bench_scenes.py --scenes sphere,clutter --brute-max-tris 0 > $OUT/scenes_$T.jsonl 2> $OUT/scenes_$T.err
echo "rc=$?"
