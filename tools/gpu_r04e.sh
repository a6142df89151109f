#!/bin/bash
# Round 4: conv kernel SQ / traffic passes (fp32 and bf16), the GAN traffic
# passes (last-4-launch fix), the VGG input-gradient test.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
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
step 300 pytest_vgg.log python -u -m pytest tests/test_gpu_gan.py -v -s --timeout 300 --timeout-method thread -k "vgg_loss_input_gradient"; ok $? || exit 1
step 600 pmc_conv_fp32.log bash tools/pmc_conv.sh "${1:-r04e}/conv_fp32" fp32 || exit 1
step 600 pmc_conv_bf16.log bash tools/pmc_conv.sh "${1:-r04e}/conv_bf16" bf16 || exit 1
step 900 pmc_gan.log bash tools/pmc_gan_r04.sh "${1:-r04e}/pmc_gan" || exit 1
echo "all steps ok"
