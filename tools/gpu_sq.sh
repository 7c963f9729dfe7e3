# SQ counter passes (each its own rocprofv3 run, --kernel-trace only) on the bench
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${TAG:-sq}
i=0
for set in "VALUBusy" "VALUUtilization" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $OUT/${T}_$i -o run --output-format csv \
      -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/${T}_$i.log 2>&1 || { echo "fail $i" > $OUT/${T}.status; exit 1; }
done
echo ok > $OUT/${T}.status
