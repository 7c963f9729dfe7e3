#!/bin/bash
# Round-2 GPU-box session: smoke, GPU tests, bench, profiles.  Every GPU step
# has its own time limit; steps are chained with && so the first failure ends
# the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:-r02}
STAGE=${2:-all}
TESTS=${3:-tests}

run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1; }
run_tests() {
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
}
run_bench() { timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; }
run_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-secondary > "$OUT/prof_$TAG.log" 2>&1
}
run_pmc() {
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$TAG" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/pmc_fetch_$TAG.log" 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write_$TAG" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > "$OUT/pmc_write_$TAG.log" 2>&1
}
case "$STAGE" in
  all) run_smoke && run_tests && run_bench && run_prof && run_pmc ;;
  tests) run_smoke && run_tests ;;
  testbench) run_smoke && run_tests && run_bench ;;
  bench) run_bench && run_prof && run_pmc ;;
  benchonly) run_bench ;;
  prof) run_prof && run_pmc ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc" > "$OUT/round_$TAG.status"
exit $rc
