#!/bin/bash
# Round-3 GPU pass: GPU suite, smoke, C2 fp32 bench, bf16 C3-shape bench, and
# (mode "prof") rocprofv3 kernel stats of the C2 bench + a roctx phase trace.
#   gpurun -- bash tools/gpu_r03.sh <tag> [prof|noprof] [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-r03}
MODE=${2:-noprof}
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
if [ -n "$3" ]; then
  step 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$3" || exit 1
else
  step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
fi
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step 300 bench.json python bench.py || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
if [ "$MODE" = prof ]; then
  step 300 prof.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-graph || exit 1
  AINP_TRACE=1 step 300 phase.log rocprofv3 --marker-trace --hip-runtime-trace --kernel-trace -f csv \
    -d "$OUT/phase" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph || exit 1
  python3 tools/phase_table.py "$OUT/phase" > "$OUT/phase_table.txt" 2>&1; cat "$OUT/phase_table.txt" | head -12
fi
echo "all steps ok"
