#!/bin/bash
# bf16 step with the routed 256x256 GEMM vs the 128x128 kernel only, then the
# C3-shape bf16 bench and the C2 bench (same box).
#   gpurun -- bash tools/gpu_ab2.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-ab2}
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
for v in 1 0; do
  step 240 ab$v.log env AINP_GEMM16_256=$v rocprofv3 --kernel-trace --stats -f csv -d "$OUT/ab$v" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
done
step 300 pytest_bf16.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bf16 or gan or dconv16" || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
step 300 bench.json python bench.py || exit 1
echo "all steps ok"
