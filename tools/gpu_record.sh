#!/bin/bash
# Round record on one box: part "tests" = the full -m gpu suite + smoke();
# part "bench" = the four bench lines (C2 fp32 headline, C3-shape bf16, GAN
# C4 / C5 bf16, each with its CPU baseline) and a rocprofv3 kernel-stats
# profile of the C2 bench.  Every GPU step has its own limit; the chain stops
# at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_record.sh <tag> tests|bench
set -o pipefail
TAG=${1:?tag}
PART=${2:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <seconds> <logfile> cmd...
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$log" | cut -c1-300
  return $rc
}
if [ "$PART" = tests ]; then
  step 1000 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
  step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
else
  step 300 bench_c2.json python bench.py || exit 1
  step 300 bench_c3.json python bench.py --dtype bf16 || exit 1
  step 400 bench_gan_c4.json python bench.py --workload gan --dtype bf16 || exit 1
  step 400 bench_gan_c5.json python bench.py --workload gan --dtype bf16 --clip-s 8 || exit 1
  step 300 prof_c2.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_c2" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
fi
echo "all steps ok"
