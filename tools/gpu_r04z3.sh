#!/bin/bash
# Round 4: the encoder's first-conv weight gradient on the main stream
# (AINP_WGRAD_LAST_MAIN): model tests, C2 / C3 A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04z3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py > "$OUT/pytest_model.log" 2>&1 || { tail -30 "$OUT/pytest_model.log"; exit 1; }
tail -2 "$OUT/pytest_model.log"
run() {  # tag dtype env...
  local tag=$1 dt=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --dtype $dt --no-cpu-baseline --steps 30 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || return 1
  python - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in 1 2 3; do
  run c2_main1_$rep fp32 AINP_WGRAD_LAST_MAIN=1 || exit 1
  run c2_main0_$rep fp32 AINP_WGRAD_LAST_MAIN=0 || exit 1
  run c3_main1_$rep bf16 AINP_WGRAD_LAST_MAIN=1 || exit 1
  run c3_main0_$rep bf16 AINP_WGRAD_LAST_MAIN=0 || exit 1
done
echo "all steps ok"
