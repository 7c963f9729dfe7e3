# variant A/B + GPU tests + phase timing in one call
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${TAG:-k}
timeout -k 10 400 python tools/variant_bench.py ${VARIANTS:-pairs fused fused4} > $OUT/variants_$T.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu_$T.log 2>&1
echo "rc=$?" > $OUT/multi_$T.status
timeout -k 10 200 python tools/phase_timing.py > $OUT/phase_$T.log 2>&1
echo "rc_phase=$?" >> $OUT/multi_$T.status
