#!/bin/bash
# Round 4: bf16 conv persistent-grid multiplier A/B (AINP_X6_OCC16 1..4) on the
# conv probe, the VGG input-gradient test, then the C3-shape bench per setting.
set -o pipefail
OUT=gpurun_out/${1:-r04f}
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
for o in 1 2 3 4; do
  AINP_X6_OCC16=$o step 120 probe_occ$o.log python tools/conv_probe.py 5 bf16 16-32,32-16,32-64 || exit 1
  cat "$OUT/probe_occ$o.log" | grep -v amdgpu.ids
done
for o in 1 2 4 1 2 4; do
  AINP_X6_OCC16=$o step 300 bench_bf16_occ$o.json python bench.py --dtype bf16 --no-cpu-baseline --no-graph --steps 30 || exit 1
done
AINP_X6_OCC16=2 step 600 pytest_bf16.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -k "bf16"; ok $? || exit 1
echo "all steps ok"
