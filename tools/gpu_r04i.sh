#!/bin/bash
# Round 4: data gradient with the fused BatchNorm-backward reduction
# (ainp_conv3x3_dgrad_bnb) and the 128-wide NTCF bridge tiles: parity tests,
# the BN probe per tile variant, then C2 / C3-shape benches fused vs separate.
set -o pipefail
OUT=gpurun_out/${1:-r04i}
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
K="bnb or bn_relu or ntcf or cast_bf16 or conv3x3"
step 600 pytest_k.log python -u -m pytest tests/test_gpu_kernels.py -v --timeout 120 --timeout-method thread -k "$K"
for t in 12864 64128; do
  AINP_NTCF_BWD_T=$t step 300 pytest_k_$t.log python -u -m pytest tests/test_gpu_kernels.py -v --timeout 120 --timeout-method thread -k "bn_relu"
done
AINP_NTCF16_T=64 step 300 pytest_k_b64.log python -u -m pytest tests/test_gpu_kernels.py -v --timeout 120 --timeout-method thread -k "cast_bf16"
step 120 bn_probe.log python tools/bn_probe.py 10 || exit 1
AINP_NTCF_BWD_T=12864 step 120 bn_probe_12864.log python tools/bn_probe.py 10 || exit 1
AINP_NTCF_BWD_T=64128 AINP_NTCF16_T=64 step 120 bn_probe_64128.log python tools/bn_probe.py 10 || exit 1
for f in bn_probe.log bn_probe_12864.log bn_probe_64128.log; do echo "-- $f"; grep -v amdgpu.ids "$OUT/$f"; done
AINP_NTCF16_T=64 step 900 pytest_model.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 > "$OUT/c2_$tag.json" 2> "$OUT/c2_$tag.err" || return 1
  env "$@" timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --no-graph --steps 30 > "$OUT/c3_$tag.json" 2> "$OUT/c3_$tag.err" || return 1
  python - "$OUT" "$tag" <<'PY'
import json, sys
out, tag = sys.argv[1:]
for k in ("c2", "c3"):
    for l in open(f"{out}/{k}_{tag}.json"):
        if l.startswith("{"):
            d = json.loads(l)
            print(f"{k} {tag}: {d['ms_per_step']} ms/step median {d['ms_per_step_median']}", flush=True)
PY
}
for rep in 1 2; do
  run sep_$rep AINP_BN_BWD_FUSED=0 AINP_NTCF16_T=64 || exit 1
  run fused_$rep AINP_BN_BWD_FUSED=1 AINP_NTCF16_T=64 || exit 1
  run fused_12864_$rep AINP_BN_BWD_FUSED=1 AINP_NTCF_BWD_T=12864 AINP_NTCF16_T=64 || exit 1
  run fused_64128_$rep AINP_BN_BWD_FUSED=1 AINP_NTCF_BWD_T=64128 AINP_NTCF16_T=64 || exit 1
done
echo "all steps ok"
