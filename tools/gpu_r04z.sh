#!/bin/bash
# Round 4 record: (A) the whole GPU suite + smoke, or (B) the benches (C2 with
# the CPU baseline, C3-shape, C4, C5), the bench's rocprofv3 kernel summary and
# the per-step kernel tables.
#   gpurun -- bash tools/gpu_r04z.sh <tag> A|B
set -o pipefail
OUT=gpurun_out/${1:-r04z}
PART=${2:-A}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -1 "$OUT/$log" | cut -c1-250
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "$PART" = A ]; then
  step 1100 pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; ok $? || exit 1
  step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
else
  step 300 pytest_gy16.log python -u -m pytest tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "gy_storage"; ok $? || exit 1
  step 400 bench.json python bench.py || exit 1
  step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
  step 300 bench_gan_c4.json python bench.py --workload gan --dtype bf16 --no-cpu-baseline || exit 1
  step 300 bench_gan_c5.json python bench.py --workload gan --dtype bf16 --clip-s 8 --no-cpu-baseline || exit 1
  step 400 bench_prof.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench_prof" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
  step 300 cnn_fp32.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_fp32" -o run -- \
    python3 tools/step_prof.py --steps 10 || exit 1
  step 300 cnn_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
  step 300 gan_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_bf16" -o run -- \
    python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 || exit 1
fi
echo "all steps ok"
