#!/bin/bash
# One GPU-box pass: GPU parity tests, the CNNBLSTM bench, the per-op timer,
# a rocprofv3 kernel-trace of the bench and the GAN bench.  Every GPU step has
# its own time limit and the chain stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh <tag> [tests|notests]
set -o pipefail
TAG=${1:-run}
TESTS=${2:-tests}
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
if [ "$TESTS" = tests ]; then
  step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
fi
step 300 bench.json python bench.py || exit 1
step 200 opbench.log python tools/cnnblstm_op_bench.py || exit 1
step 300 prof.log rocprofv3 --kernel-trace --stats -f csv rocpd -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
step 300 bench_gan.json python bench.py --workload gan || exit 1
echo "all steps ok"
