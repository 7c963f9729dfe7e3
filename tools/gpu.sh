#!/bin/bash
# One GPU-box session (gpurun): tools/gpu.sh TAG STAGE [STAGE ...]
#
# Every stage that touches the GPU runs under its own time limit and the
# stages are chained: the first failure ends the call (no retries).  Outputs
# go to gpurun_out/<stage>_<TAG>.*; copy what is to be judged into profiles/.
#
# Stages:
#   smoke        __graft_entry__.smoke()
#   tests        pytest -m gpu ($TESTS, default tests; $PYTEST_K for -k)
#   bench        bench.py (full JSON line)
#   benchq       bench.py --no-secondary --no-cpu-baseline
#   benchd       bench.py exactly as the driver runs it (--gpus 1 --steps 20 --warmup 5)
#   benchrep     the driver's form three times back to back (run-to-run spread in one box)
#   benchsteps   headline only (--no-secondary --no-cpu-baseline) at 20 / 60 / 200 steps, warmup 5
#   prof         rocprofv3 --kernel-trace --stats of the C2 headline (no secondary lines)
#   pmc          FETCH_SIZE / WRITE_SIZE passes of the C2 headline (separate runs)
#   sq           SQ counter passes of the C2 headline
#   attr         memory-side request classes of the C2 headline (atomics vs reads vs writes, TCC/TCP)
#   valumix      VALU instruction-mix counter passes of the C2 headline
#   uprof        kernel stats + FETCH/WRITE/TCC passes of the unbounded legs (tools/unbounded_prof.py)
#   usq          SQ counter passes of the unbounded legs
#   ulds / lds   LDS bank-conflict counters of the unbounded legs / the C2 headline
#   nsprof       rocprofv3 --kernel-trace --stats of the north-star scene (BVH instances)
#   nspmc        FETCH/WRITE + SQ counter passes of the north-star scene
#   scenes       tools/bench_scenes.py ($SCENES, default all)
#   c5           tools/bench_c5.py
#   graph        tools/bench_graph.py (createGraph at the reference config)
#   variants     tools/variant_bench.py $VARIANTS ($VB_ONLY scenes; IPT_VB_* passed through)
#   phase        tools/phase_timing.py
#   stats        tools/bvh_stats.py with the IPT_BVH_STATS variant library ($SCENES)
#   multirank    2-rank gloo rehearsal of bench.py on the one GPU
#   scaling      tools/launch_scaling.py (fixed cost per launch: C2 shares 1/1 .. 1/64)
#   workflow     tools/workflow_at_size.py (pipeline all --n 100 + optimize --n 100)
#   graphprof    rocprofv3 --kernel-trace --stats of createGraph at the reference config (tools/graph_prof.py)
#   pipeab       tools/pipeline_ab.py (consecutive frames on one stream vs two)
#   adjpmc       tools/adj_pmc.py: kernel stats + FETCH/WRITE/TCC/TCP passes of the C2 fused render and adjoint,
#                for the default library, $ADJ_VARIANT (a lib/variants build) and the 5-wave adjoint (IPT_ADJW=0)
#   counters     rocprofv3 -L (the counters this box offers)
#   vtests       pytest -m gpu ($VTESTS, -k "$VT_K") against lib/variants/libipt_$VT_VARIANT.so (IPT_AMD_LIB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
T=${1:?usage: tools/gpu.sh TAG STAGE...}
shift

pmc_passes() {  # pmc_passes NAME CMD... : one rocprofv3 run per counter set in $SETS (newline-separated)
  local name=$1; shift
  local i=0
  while IFS= read -r set; do
    [ -z "$set" ] && continue
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/${name}_${T}_$i" -o run --output-format csv \
        -- "$@" > "$OUT/${name}_${T}_$i.log" 2>&1 || return 1
  done <<< "$SETS"
}
SQ_SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS
SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
VALUBusy
VALUUtilization"
ATTR_SETS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum
TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum
TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
TCC_HIT_sum TCC_MISS_sum"
MIX_SETS="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64
SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"
BENCHQ=(python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-secondary)
NS=(python3 "$R/tools/bench_scenes.py" --scenes northstar --brute-max-tris 0)
UP=(python3 "$R/tools/unbounded_prof.py")

run() {
  case "$1" in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$T.log" 2>&1 ;;
    tests) timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v --maxfail=5 --timeout 300 \
               --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu_$T.log" 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > "$OUT/bench_$T.json" 2> "$OUT/bench_$T.err" ;;
    benchd) timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/benchd_$T.json" 2> "$OUT/benchd_$T.err" ;;
    benchsteps) for k in 20 60 200 20; do
                  timeout -k 10 300 python3 bench.py --steps $k --warmup 5 --no-secondary --no-cpu-baseline \
                      >> "$OUT/benchsteps_$T.jsonl" 2>> "$OUT/benchsteps_$T.err" || return 1
                done ;;
    benchrep) for k in 1 2 3; do
                timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/benchrep_${T}_$k.json" \
                    2> "$OUT/benchrep_${T}_$k.err" || return 1
              done ;;
    benchq) timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > "$OUT/benchq_$T.json" 2> "$OUT/benchq_$T.err" ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$T" -o run --output-format csv \
              -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/prof_$T.log" 2>&1 ;;
    pmc) SETS=$'FETCH_SIZE\nWRITE_SIZE' pmc_passes pmc "${BENCHQ[@]}" ;;
    sq) SETS=$SQ_SETS pmc_passes sq "${BENCHQ[@]}" ;;
    attr) SETS=$ATTR_SETS pmc_passes attr "${BENCHQ[@]}" ;;
    uprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/uprof_$T" -o run --output-format csv \
               -- "${UP[@]}" > "$OUT/uprof_$T.log" 2>&1 &&
           SETS=$'FETCH_SIZE\nWRITE_SIZE\nTCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum' pmc_passes upmc "${UP[@]}" --steps 2 ;;
    valumix) SETS=$MIX_SETS pmc_passes valumix "${BENCHQ[@]}" ;;
    usq) SETS=$SQ_SETS pmc_passes usq "${UP[@]}" --steps 2 ;;
    ulds) SETS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" pmc_passes ulds "${UP[@]}" --steps 2 ;;
    lds) SETS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" pmc_passes lds "${BENCHQ[@]}" ;;
    nsprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/nsprof_$T" -o run --output-format csv \
                -- "${NS[@]}" --steps 10 > "$OUT/nsprof_$T.log" 2>&1 ;;
    nspmc) SETS=$'FETCH_SIZE\nWRITE_SIZE\n'"$SQ_SETS" pmc_passes nspmc "${NS[@]}" --steps 2 ;;
    scenes) timeout -k 10 300 python tools/bench_scenes.py ${SCENES:+--scenes $SCENES} > "$OUT/scenes_$T.jsonl" 2> "$OUT/scenes_$T.err" ;;
    c5) timeout -k 10 300 python tools/bench_c5.py > "$OUT/c5_$T.json" 2> "$OUT/c5_$T.err" ;;
    graph) timeout -k 10 300 python tools/bench_graph.py > "$OUT/graph_$T.json" 2> "$OUT/graph_$T.err" ;;
    variants) IPT_VB_ONLY=${VB_ONLY:-$IPT_VB_ONLY} timeout -k 10 600 python tools/variant_bench.py ${VARIANTS:-base} \
                  > "$OUT/variants_$T.log" 2>&1 ;;
    phase) timeout -k 10 300 python tools/phase_timing.py > "$OUT/phase_$T.log" 2>&1 ;;
    stats) IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_stats.so timeout -k 10 300 \
               python tools/bvh_stats.py ${SCENES:+--scenes $SCENES} --out "$OUT/stats_$T.json" > "$OUT/stats_$T.log" 2>&1 ;;
    multirank) IPT_BENCH_DEVICE=0 IPT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
                   --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 \
                   --warmup 4 > "$OUT/bench_2rank_$T.json" 2> "$OUT/bench_2rank_$T.err" ;;
    scaling) timeout -k 10 300 python tools/launch_scaling.py > "$OUT/scaling_$T.jsonl" 2> "$OUT/scaling_$T.err" ;;
    workflow) timeout -k 10 1000 python -u tools/workflow_at_size.py --out "$OUT/workflow_$T.json" > "$OUT/workflow_$T.log" 2>&1 ;;
    graphprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/graphprof_$T" -o run --output-format csv \
                   -- python3 "$R/tools/graph_prof.py" --steps 20 > "$OUT/graphprof_$T.log" 2>&1 ;;
    adjpmc) local sets=$'FETCH_SIZE\nWRITE_SIZE\nTCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_MISS_sum\nTCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum'
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/adjstats_$T" -o run --output-format csv \
                -- python3 "$R/tools/adj_pmc.py" --steps 10 > "$OUT/adjstats_$T.log" 2>&1 &&
            SETS=$sets pmc_passes adjpmc_new python3 "$R/tools/adj_pmc.py" &&
            ( export IPT_ADJW=0; SETS=$sets pmc_passes adjpmc_five python3 "$R/tools/adj_pmc.py" --no-fwd ) &&
            if [ -n "$ADJ_VARIANT" ]; then
              ( export IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_$ADJ_VARIANT.so
                SETS=$sets pmc_passes adjpmc_var python3 "$R/tools/adj_pmc.py" ) &&
              ( export IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_$ADJ_VARIANT.so
                timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/adjstats_var_$T" -o run --output-format csv \
                    -- python3 "$R/tools/adj_pmc.py" --steps 10 > "$OUT/adjstats_var_$T.log" 2>&1 )
            fi ;;
    vtests) IPT_AMD_LIB=$R/inverse_path_tracer_amd/lib/variants/libipt_$VT_VARIANT.so timeout -k 10 600 \
                python -u -m pytest ${VTESTS:-tests} -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
                -p no:cacheprovider ${VT_K:+-k "$VT_K"} > "$OUT/pytest_gpu_${VT_VARIANT}_$T.log" 2>&1 ;;
    counters) timeout -k 10 120 rocprofv3 -L > "$OUT/counters_$T.txt" 2>&1 ;;
    pipeab) timeout -k 10 300 python tools/pipeline_ab.py > "$OUT/pipeab_$T.log" 2>&1 ;;
    *) echo "unknown stage $1" >&2; return 2 ;;
  esac
}

rc=0
for s in "$@"; do
  run "$s" || { rc=$?; echo "stage $s failed rc=$rc" > "$OUT/status_$T"; break; }
done
[ $rc -eq 0 ] && echo "ok: $*" > "$OUT/status_$T"
exit $rc
