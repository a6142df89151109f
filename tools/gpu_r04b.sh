#!/bin/bash
# Round 4: generator-backward tests + the VGG input-gradient diagnostic.
set -o pipefail
OUT=gpurun_out/${1:-r04b}
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
step 300 vgg_diag.log python tools/vgg_grad_diag.py; ok $? || exit 1
step 600 pytest_gbwd.log python -u -m pytest tests/test_gpu_gan.py -v -s --timeout 300 --timeout-method thread -k "gen_bwd_kernels or vgg_loss_input_gradient or generator_training_step or generator_small or generator_full or gan_step_matches_oracle" || exit 1
echo "all steps ok"
