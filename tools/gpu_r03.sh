#!/bin/bash
# Round-3 GPU pass: GPU suite, smoke, C2 fp32 bench, bf16 C3-shape bench.
#   gpurun -- bash tools/gpu_r03.sh <tag> [quick]
set -o pipefail
OUT=gpurun_out/${1:-r03}
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
step 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step 300 bench.json python bench.py || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
echo "all steps ok"
