#!/bin/bash
# Round 4: the bf16 64 -> 32 data gradient on the persistent x6p kernel
# (AINP_X6P_DG64=1) vs the 8-row tiled kernel: parity with it on, C3 A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04y}
mkdir -p "$OUT"
export TMPDIR=/tmp
AINP_X6P_DG64=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "conv3x3" > "$OUT/pytest_k.log" 2>&1 || { tail -30 "$OUT/pytest_k.log"; exit 1; }
tail -2 "$OUT/pytest_k.log"
AINP_X6P_DG64=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py -k "bf16" > "$OUT/pytest_model.log" 2>&1 || { tail -30 "$OUT/pytest_model.log"; exit 1; }
tail -2 "$OUT/pytest_model.log"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --steps 30 \
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
  run c3_dg64_$rep AINP_X6P_DG64=1 || exit 1
  run c3_tiled_$rep AINP_X6P_DG64=0 || exit 1
done
AINP_X6P_DG64=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/step" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 > "$OUT/step.log" 2>&1 || exit 1
grep "ms/step" "$OUT/step.log"
echo "all steps ok"
