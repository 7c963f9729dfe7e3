set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python tools/variant_bench.py cur cur4 nospec_b5 abl_norm abl_trig abl_dp abl_all > $OUT/variants_f.log 2>&1
echo rc=$? > $OUT/cmd.status
