#!/bin/bash
# Round-2 late pass: full -m gpu suite, then the bf16 benches (C3 shape, C4 GAN).
#   gpurun -- bash tools/gpu_r02s.sh <tag> [fp32]
set -o pipefail
OUT=gpurun_out/${1:-r02s}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$log"
  return $rc
}
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
if [ "${2:-}" = fp32 ]; then
  step 300 bench.json python bench.py || exit 1
fi
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
step 300 bench_gan_bf16.json python bench.py --workload gan --dtype bf16 --no-cpu-baseline || exit 1
echo "all steps ok"
