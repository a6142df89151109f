#!/bin/bash
# Round 5: channel-last conv path -- kernel tests, the model step test, then
# C2 / C3-shape bench A/B (AINP_CL=1 vs 0) on one box.
#   gpurun -- bash tools/gpu_cl_check.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-clcheck}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_cl.py > "$OUT/pytest_cl.log" 2>&1 || { tail -40 "$OUT/pytest_cl.log"; exit 1; }
tail -2 "$OUT/pytest_cl.log"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "conv3x3 or small_wgrad" > "$OUT/pytest_conv.log" 2>&1 || { tail -40 "$OUT/pytest_conv.log"; exit 1; }
tail -2 "$OUT/pytest_conv.log"
run() {  # tag dtype env...
  local tag=$1 dt=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --dtype $dt --no-cpu-baseline --steps 20 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || return 1
  python - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in 1 2; do
  run c2_cl1_$rep fp32 AINP_CL=1 || exit 1
  run c2_cl0_$rep fp32 AINP_CL=0 || exit 1
  run c3_cl1_$rep bf16 AINP_CL=1 || exit 1
  run c3_cl0_$rep bf16 AINP_CL=0 || exit 1
done
echo "all steps ok"
