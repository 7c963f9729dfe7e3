set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python tools/variant_bench.py ${VARIANTS:-flat flat4 flat6 tab nospec_b5} > $OUT/variants_${TAG:-g}.log 2>&1
echo rc=$? > $OUT/cmd.status
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu_${TAG:-g}.log 2>&1
echo rc2=$? >> $OUT/cmd.status
