#!/bin/bash
# Round 4: bf16 storage of the pre-BN conv outputs (AINP_CONV_X16 / _Y16,
# AINP_BN_Y16; cnnblstm.Y16): parity (kernels bit-exact vs fp32 reads of the
# same values; the bf16 C2 gate against the re-generated emulation), the model
# and DP suites, then the C3-shape bench with and without it.
set -o pipefail
OUT=gpurun_out/${1:-r04k}
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
step 300 pytest_k.log python -u -m pytest tests/test_gpu_kernels.py -v --timeout 120 --timeout-method thread -k "activation_storage or read_bf16_y or bf16_dy or bf16_output or refused or bn_relu or conv3x3 or cast_bf16"; ok $? || exit 1
step 900 pytest_model.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dist.py -v -s --timeout 300 --timeout-method thread; ok $? || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --no-graph --steps 30 > "$OUT/c3_$tag.json" 2> "$OUT/c3_$tag.err" || return 1
  python - "$OUT" "$tag" <<'PY'
import json, sys
out, tag = sys.argv[1:]
for l in open(f"{out}/c3_{tag}.json"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"c3 {tag}: {d['ms_per_step']} ms/step median {d['ms_per_step_median']}", flush=True)
PY
}
for rep in 1 2 3; do
  run y0_$rep AINP_Y16=0 || exit 1
  run y1_$rep AINP_Y16=1 || exit 1
done
echo "all steps ok"
