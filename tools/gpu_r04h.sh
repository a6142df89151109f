#!/bin/bash
# Round 4: BLSTM backward issue order (AINP_MAIN_FIRST) and HIP stream
# priorities (AINP_MAIN_PRIO / AINP_SIDE_PRIO) A/B on the C2 and C3-shape
# benches, after the model / DP tests under the new default order.
set -o pipefail
OUT=gpurun_out/${1:-r04h}
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
step 120 bn_probe.log python tools/bn_probe.py 10 || exit 1
grep -v amdgpu.ids "$OUT/bn_probe.log"
step 900 pytest_model.log python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread || exit 1
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
  run mf0_$rep AINP_MAIN_FIRST=0 || exit 1
  run mf1_$rep AINP_MAIN_FIRST=1 || exit 1
  run mf1_mainhi_$rep AINP_MAIN_FIRST=1 AINP_MAIN_PRIO=-1 || exit 1
  run mf1_sidelo_$rep AINP_MAIN_FIRST=1 AINP_SIDE_PRIO=1 || exit 1
done
grep -h "priority range" "$OUT"/*.json | head -2
echo "all steps ok"
