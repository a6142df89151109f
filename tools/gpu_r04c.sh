#!/bin/bash
# Round 4: per-step kernel tables (C2 fp32, C3-shape bf16, C4 / C5 bf16 GAN)
# and the GAN roofline kernels' FETCH/WRITE passes on in-step operands.
set -o pipefail
OUT=gpurun_out/${1:-r04c}
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
step 300 cnn_fp32.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_fp32" -o run -- \
  python3 tools/step_prof.py --steps 10 || exit 1
step 300 cnn_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
step 300 gan_c4.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_c4" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 10 --dtype bf16 || exit 1
step 300 gan_c5.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_c5" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 10 --dtype bf16 --clip-s 8 || exit 1
step 900 pmc_gan.log bash tools/pmc_gan_r04.sh "${1:-r04c}/pmc_gan" || exit 1
echo "all steps ok"
