#!/bin/bash
# Round 4: generator-backward tests, the per-step kernel tables (C2, C3-shape,
# C4, C5) and the GAN roofline kernels' FETCH/WRITE passes.
set -o pipefail
OUT=gpurun_out/${1:-r04d}
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
step 600 pytest_gbwd.log python -u -m pytest tests/test_gpu_gan.py -v -s --timeout 300 --timeout-method thread -k "gen_bwd_kernels or vgg_loss_input_gradient or generator_training_step or generator_small or generator_full or gan_step_matches_oracle or full_size_gan_step"; ok $? || exit 1
step 300 cnn_fp32.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_fp32" -o run -- \
  python3 tools/step_prof.py --steps 10 || exit 1
step 300 cnn_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
step 300 gan_c4.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_c4" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 10 --dtype bf16 || exit 1
step 300 gan_c5.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_c5" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 10 --dtype bf16 --clip-s 8 || exit 1
step 900 pmc_gan.log bash tools/pmc_gan_r04.sh "${1:-r04d}/pmc_gan" || exit 1
echo "all steps ok"
