#!/bin/bash
# Round-2 GPU pass: selected tests (or the whole -m gpu suite), the bench and a
# rocprofv3 kernel trace of it.  Each step has its own time limit; the chain
# stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_r02.sh <tag> <pytest -k expr|all|none> [bench|nobench] [prof|noprof]
set -o pipefail
TAG=${1:-run}
SEL=${2:-all}
BENCH=${3:-bench}
PROF=${4:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <seconds> <logfile> cmd...
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$log"
  return $rc
}
if [ "$SEL" = all ]; then
  step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
elif [ "$SEL" != none ]; then
  step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$SEL" || exit 1
fi
if [ "$BENCH" = bench ]; then
  step 300 bench.json python bench.py || exit 1
fi
if [ "$PROF" = prof ]; then
  step 300 prof.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
fi
echo "all steps ok"
