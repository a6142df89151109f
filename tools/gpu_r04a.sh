#!/bin/bash
# Round 4, first pass: the DP tests (device collectives, fused layer-0 pair
# under DP, G-loss fail-fast), the tightened bf16 gates, `bench.py --gpus 2`
# spawning its own ranks (gloo on the box's one GPU), the C2 / C3-shape
# benches, then the new generator-backward tests.
#   gpurun -- bash tools/gpu_r04a.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r04a}
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
# an assertion failure (rc 1) is data; a crash / timeout ends the call
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
step 900 pytest_dist.log python -u -m pytest tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread; ok $? || exit 1
step 600 pytest_bf16gates.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_gan.py -v -s --timeout 300 --timeout-method thread -k "bf16_c2_batch32 or bf16_tracks_reference"; ok $? || exit 1
AINP_DIST_BACKEND=gloo step 400 dp2_spawn.json python bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline --no-graph; ok $? || exit 1
step 300 bench.json python bench.py --no-cpu-baseline --no-graph || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline --no-graph || exit 1
step 600 pytest_gbwd.log python -u -m pytest tests/test_gpu_gan.py -v -s --timeout 300 --timeout-method thread -k "gen_bwd_kernels or vgg_loss_input_gradient or generator_training_step or generator_small or generator_full or gan_step_matches_oracle" || exit 1
echo "all steps ok"
