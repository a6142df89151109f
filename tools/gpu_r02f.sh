#!/bin/bash
# Closing pass after the bf16 projection split: GPU suite, smoke, C2 + bf16 benches,
# rocprofv3 stats of the bf16 bench, PMC traffic of the split bf16 projection.
#   gpurun -- bash tools/gpu_r02f.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r02f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -1 "$OUT/$log" | cut -c1-300
  return $rc
}
step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step 300 bench.json python bench.py || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
step 300 prof_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_bf16" -o run -- \
  python3 bench.py --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
step 400 pmc_bf16.log bash tools/pmc_gemm.sh ${1:-r02f}/pmc_bf16 bf16 || exit 1
echo "all steps ok"
